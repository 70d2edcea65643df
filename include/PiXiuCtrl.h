// PiXiuCtrl.h — source-compatible C++ facade of the reference's PiXiuCtrl
// (reference src/proj/PiXiuCtrl.h:7-26, README.md:100-150), implemented over the
// C ABI in pixiu_amd.h.  Header-only; link against libpixiu_amd.so.
//
// Client code written for the reference keeps compiling:
//
//     PiXiuCtrl ctrl; ctrl.init_prop();
//     ctrl.setitem((uint8_t *)k, klen, (uint8_t *)v, vlen);
//     PXSGen *gen = ctrl.getitem((uint8_t *)k, klen);
//     uint8_t rv; while (gen->operator()(rv)) putchar(rv);
//     PXSGen_free(gen);
//     ctrl.free_prop();
//
// including the CLI's `ctrl.st.cbt_chunk->getitem(ctrl.st.local_chunk.used_num - 1)->len`
// (main.cpp:67).  Semantics are the reference's single instance (one shard);
// getitem and iter stream the compat expansion (PXSGen byte-for-byte).  Generators are
// lazy: getitem only looks the record up and expands it (<= 64 KiB) at the first pull;
// iter expands its records kIterWindow at a time as the caller advances, so host memory
// stays bounded whatever the prefix matches.  A generator pulled after free_prop() or
// init_prop() yields nothing and reports PX_EINVAL in its `status` (an extension; the
// reference's generators dangle there).  reinsert(PiXiuChunk *&) compacts a closed
// slot-full chunk (PiXiuCtrl.cpp:88-114); chunk_at(seq) names one (an extension: the
// reference reaches its chunks only through its internals).
//
// setitem is write-behind (px_opts.defer_bytes = kDeferBytes): a call queues its record
// and returns the reference's value (0, or CBT_SET_REPLACE for a key already stored or
// queued) at once; the queue is stored in one batch once kDeferBytes raw bytes are
// pending, or before any read (getitem, contains, iter, delitem, the chunk view,
// st.local_chunk.used_num).  So a stream of one-record calls costs one batch per
// kDeferBytes instead of one suffix-array pass over the live chunk per call, with the
// same stored bytes (include/pixiu_amd.h px_flush).
#ifndef PIXIU_CTRL_FACADE_H
#define PIXIU_CTRL_FACADE_H

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <memory>
#include <vector>

#include "pixiu_amd.h"

#define CBT_SET_REPLACE 1
#define CBT_DEL_NOT_FOUND 1
#define PXSG_MAX_TO 65535
#define PXC_STR_NUM 65535

struct PiXiuStr {  // compressed record as the reference lays it out (PiXiuStr.h:61-64)
    uint16_t len;
    uint8_t data[1];
};

// the context a PiXiuCtrl's generators expand through: free_prop / init_prop bump the
// epoch (and free_prop clears ctx), so a generator outliving them yields nothing instead
// of reading a freed context or a slot that now holds another record
struct PxHandle {
    px_ctx *ctx = nullptr;
    uint64_t epoch = 0;
};

// PiXiuStr::parse(0, PXSG_MAX_TO)'s generator: the record is addressed at getitem time and
// expanded on the GPU at the first pull (or handed over already expanded by CBTGen).
struct PXSGen {
    std::shared_ptr<PxHandle> h;
    uint64_t epoch = 0;
    px_rec rec{};
    bool ready = false;
    int status = PX_OK;  // extension: PX_OK, or why the expansion failed (then nothing is yielded)
    std::vector<uint8_t> buf;
    size_t cur = 0;

    bool operator()(uint8_t &rv) {
        if (!ready) expand();
        if (cur >= buf.size()) return false;
        rv = buf[cur++];
        return true;
    }

    // PiXiuStr.h:200-211: drain, keep visible bytes 33..126, NUL-terminate, free the gen
    char *consume_repr(void);

  private:
    void expand() {
        ready = true;
        if (!h || !h->ctx || h->epoch != epoch) {  // free_prop / init_prop since getitem
            status = PX_EINVAL;
            buf.clear();
            return;
        }
        // a compat expansion is at most PXSG_MAX_TO + 1 bytes (the over-yield of a range
        // ending inside a 251 pair); the call reports the exact need if it is short
        buf.resize(PXSG_MAX_TO + 1024);
        uint64_t off = 0, need = 0;
        uint32_t len = 0, st = PX_EINVAL;
        int rc = px_parse_batch(h->ctx, 1, &rec, PX_COMPAT, buf.data(), buf.size(), 0, &off, &len, &st, &need);
        if (rc == PX_ESPACE) {
            buf.resize(need);
            st = PX_EINVAL;
            rc = px_parse_batch(h->ctx, 1, &rec, PX_COMPAT, buf.data(), buf.size(), 0, &off, &len, &st, &need);
        }
        if (rc != PX_OK || st != PX_OK) {
            status = rc != PX_OK ? rc : (int)st;
            buf.clear();
            return;
        }
        buf.erase(buf.begin(), buf.begin() + (long)off);
        buf.resize(len);
        buf.shrink_to_fit();
    }
};

// PiXiuCtrl::iter's generator (CritBitTree.h:134-157): the matching records in yield order,
// expanded kIterWindow at a time, one batch per window, as the caller advances.
struct CBTGen {
    static constexpr uint32_t kIterWindow = 64;
    std::shared_ptr<PxHandle> h;
    uint64_t epoch = 0;
    std::vector<px_rec> recs;
    std::vector<std::vector<uint8_t>> win;  // expansions of recs[base .. base + win.size())
    std::vector<int> win_st;                // and their statuses
    size_t cur = 0, base = 0;

    bool operator()(PXSGen *&rv) {
        if (cur >= recs.size()) return false;
        if (cur >= base + win.size()) fill(cur);
        rv = new PXSGen();
        rv->h = h;
        rv->epoch = epoch;
        rv->rec = recs[cur];
        rv->ready = true;
        rv->status = win_st[cur - base];
        rv->buf = std::move(win[cur - base]);
        ++cur;
        return true;
    }

  private:
    void fill(size_t at) {
        const uint32_t n = (uint32_t)std::min<size_t>(kIterWindow, recs.size() - at);
        base = at;
        win.assign(n, std::vector<uint8_t>());
        win_st.assign(n, PX_EINVAL);  // (a window that cannot be expanded yields failed generators)
        if (!h || !h->ctx || h->epoch != epoch) return;
        std::vector<uint8_t> out((size_t)n * (PXSG_MAX_TO + 1024));
        std::vector<uint64_t> off(n);
        std::vector<uint32_t> len(n), status(n, PX_EINVAL);
        uint64_t need = 0;
        int rc = px_parse_batch(h->ctx, n, recs.data() + at, PX_COMPAT, out.data(), out.size(), 0, off.data(),
                                len.data(), status.data(), &need);
        if (rc == PX_ESPACE) {
            out.resize(need);
            std::fill(status.begin(), status.end(), (uint32_t)PX_EINVAL);
            rc = px_parse_batch(h->ctx, n, recs.data() + at, PX_COMPAT, out.data(), out.size(), 0, off.data(),
                                len.data(), status.data(), &need);
        }
        for (uint32_t i = 0; i < n; ++i) {
            // a failed call leaves its per-record statuses unwritten: every record fails with it
            win_st[i] = rc != PX_OK && rc != (int)status[i] && status[i] == PX_OK ? rc : (int)status[i];
            if (win_st[i] == PX_OK) win[i].assign(out.begin() + (long)off[i], out.begin() + (long)(off[i] + len[i]));
        }
    }
};

inline void PXSGen_free(PXSGen *gen) { delete gen; }
inline void CBTGen_free(CBTGen *gen) { delete gen; }

inline char *PXSGen::consume_repr(void) {
    std::vector<char> out;
    uint8_t rv;
    while ((*this)(rv))
        if (33 <= rv && rv <= 126) out.push_back((char)rv);
    char *s = (char *)malloc(out.size() + 1);
    if (!out.empty()) memcpy(s, out.data(), out.size());
    s[out.size()] = '\0';
    PXSGen_free(this);
    return s;
}

struct PiXiuCtrl;

// The part of the reference's SuffixTree / PiXiuChunk that client code touches.
struct PiXiuChunk {
    PiXiuCtrl *owner = nullptr;
    uint32_t chunk = 0;
    std::vector<std::vector<uint8_t>> cache;
    PiXiuStr *getitem(int idx);
};

// PiXiuLocalChunk::used_num (the live chunk's record count, main.cpp:67): reading it
// stores the write-behind queue first, so it counts every record set so far
struct UsedNum {
    PiXiuCtrl *owner = nullptr;
    uint16_t n = 0;
    operator uint16_t() const;
};

struct PiXiuLocalChunk {
    UsedNum used_num;
};

struct SuffixTree {
    PiXiuChunk *cbt_chunk = nullptr;
    PiXiuLocalChunk local_chunk;
};

struct CritBitTree {};

struct PiXiuCtrl {
    static constexpr uint32_t kDeferBytes = 8u << 20;  // write-behind queue of setitem (raw bytes)
    CritBitTree cbt;
    SuffixTree st;
    px_ctx *ctx = nullptr;
    PiXiuChunk chunk_view;
    int device = 0;

    // PiXiuCtrl::setitem (PiXiuCtrl.cpp:12-47).  k_len == v_len == 0: k is a ready
    // PiXiuStr doc (the reinsert path, PiXiuCtrl.cpp:39-40), stored as it is; `reinsert`
    // skips the Glob_Reinsert_Chunk trigger (:26-29).  Returns 0, CBT_SET_REPLACE, or
    // -px_status for an input the reference would assert on.
    int setitem(uint8_t k[], int k_len, uint8_t v[], int v_len, bool reinsert = false) {
        px_set_result r;
        int rc;
        if (!k_len && !v_len) {
            if (!k) return -PX_EINVAL;
            const PiXiuStr *doc = reinterpret_cast<const PiXiuStr *>(k);
            uint64_t doff[2] = {0, doc->len};
            rc = px_set_docs(ctx, 1, doc->data, doff, 0, reinsert ? 1 : 0, &r);
        } else if (!k_len) {
            return -PX_EINVAL;  // (the reference asserts k_len, PiXiuCtrl.cpp:42)
        } else {
            uint64_t koff[2] = {0, (uint64_t)k_len}, voff[2] = {0, (uint64_t)(v_len > 0 ? v_len : 0)};
            uint8_t dummy = 0;
            rc = px_set_batch(ctx, 1, k, koff, v ? v : &dummy, voff, 0, &r);
        }
        if (rc != PX_OK) return -rc;
        // this record is accepted (stored or queued): its bookkeeping first, then an earlier
        // queued record's failure, if one is still unreported, is returned in its place
        if (r.chunk == PX_PENDING) {
            pending = true;
        } else {
            pending = false;
            apply(r);
        }
        if (flush_rc != PX_OK) {
            const int f = flush_rc;
            flush_rc = PX_OK;
            return -f;
        }
        return (int)r.replaced;
    }

    bool contains(uint8_t k[], int k_len) {
        uint64_t off[2] = {0, (uint64_t)k_len};
        uint32_t res = 0;
        return px_contains_batch(ctx, 1, k, off, &res) == PX_OK && res;
    }

    // PiXiuCtrl::getitem (PiXiuCtrl.cpp:59-61): NULL for a missing key; the record is
    // expanded when the generator is first pulled
    PXSGen *getitem(uint8_t k[], int k_len) {
        uint64_t koff[2] = {0, (uint64_t)k_len};
        px_rec r;
        uint32_t status = 0;
        if (px_locate_batch(ctx, 1, k, koff, &r, &status) != PX_OK || status != PX_OK) return nullptr;
        PXSGen *g = new PXSGen();
        g->h = h;
        g->epoch = h->epoch;
        g->rec = r;
        return g;
    }

    // PiXiuCtrl::iter (PiXiuCtrl.cpp:71-75): NULL for an empty tree
    CBTGen *iter(uint8_t prefix[], int prefix_len) {
        uint32_t n = 0;
        std::vector<px_rec> recs(64);
        int rc = px_iter(ctx, prefix, (uint64_t)(prefix_len > 0 ? prefix_len : 0), recs.data(), (uint32_t)recs.size(), &n);
        if (rc == PX_ESPACE) {
            recs.resize(n);
            rc = px_iter(ctx, prefix, (uint64_t)(prefix_len > 0 ? prefix_len : 0), recs.data(), n, &n);
        }
        if (rc != PX_OK) return nullptr;
        CBTGen *g = new CBTGen();
        g->h = h;
        g->epoch = h->epoch;
        recs.resize(n);
        g->recs = std::move(recs);
        return g;
    }

    int delitem(uint8_t k[], int k_len) {
        uint64_t off[2] = {0, (uint64_t)k_len};
        uint32_t res = CBT_DEL_NOT_FOUND;
        px_del_batch(ctx, 1, k, off, &res);
        return (int)res;
    }

    void init_prop(void) {
        if (!ctx) {
            px_opts o;
            memset(&o, 0, sizeof o);
            o.device = device;
            o.records_per_shard = 0;  // one shard: the reference's single instance
            o.defer_bytes = kDeferBytes;
            ctx = px_open(&o);
        } else {
            px_reset(ctx);
        }
        if (!h) h = std::make_shared<PxHandle>();
        h->ctx = ctx;
        h->epoch++;
        pending = false;
        flush_rc = PX_OK;
        chunk_view = PiXiuChunk();
        chunk_view.owner = this;
        closed.clear();
        st.cbt_chunk = &chunk_view;
        st.local_chunk.used_num.owner = this;
        st.local_chunk.used_num.n = 0;
    }

    void free_prop(void) {
        if (ctx) px_close(ctx);  // (drops the write-behind queue, as the reference frees everything)
        ctx = nullptr;
        if (h) {
            h->ctx = nullptr;
            h->epoch++;
        }
        pending = false;
        st.cbt_chunk = nullptr;
        closed.clear();
    }

    // PiXiuCtrl::reinsert (PiXiuCtrl.cpp:88-114): compacts a closed slot-full chunk and, as
    // the reference, clears the caller's pointer.  Other chunks (the live one, or one closed
    // by the pool count, on which the reference dereferences NULL) are left as they are.
    void reinsert(PiXiuChunk *&chunk) {
        if (!chunk || !ctx) return;
        sync_pending();
        if (px_reinsert(ctx, 0, chunk->chunk) == PX_OK) {
            closed.erase(chunk->chunk);
            chunk = nullptr;
        }
    }

    // extension: the chunk with sequence number `seq` (0 = the first), for reinsert
    PiXiuChunk *chunk_at(uint32_t seq) {
        sync_pending();
        if (seq == chunk_view.chunk) return &chunk_view;
        auto &p = closed[seq];
        if (!p) {
            p.reset(new PiXiuChunk());
            p->owner = this;
            p->chunk = seq;
        }
        return p.get();
    }

    // stores the write-behind queue and brings the live-chunk view up to date.  A failure
    // (a queued record could not be stored) is kept and returned, as -status, by the next
    // setitem -- the call whose record would otherwise be missing silently -- or by flush()
    void sync_pending() {
        if (!pending || !ctx) return;
        pending = false;
        px_set_result last;
        memset(&last, 0xff, sizeof last);  // (chunk 0xffffffff: nothing placed)
        const int rc = px_flush(ctx, &last);
        if (rc != PX_OK && flush_rc == PX_OK) flush_rc = rc;
        apply(last);
    }

    // extension: store the write-behind queue now; PX_OK or the first failure since the last
    // report (a record queued by an earlier setitem that could not be stored)
    int flush() {
        sync_pending();
        if (ctx) {
            const int rc = px_flush(ctx, nullptr);
            if (rc != PX_OK && flush_rc == PX_OK) flush_rc = rc;
        }
        const int rc = flush_rc;
        flush_rc = PX_OK;
        return rc;
    }

  private:
    void apply(const px_set_result &r) {
        if (r.chunk == 0xffffffffu) return;  // (not placed)
        if (r.chunk != chunk_view.chunk) {   // chunk rotation (PiXiuCtrl.cpp:13-25)
            chunk_view.chunk = r.chunk;
            chunk_view.cache.clear();
        }
        st.local_chunk.used_num.n = (uint16_t)(r.idx + 1);
    }
    std::shared_ptr<PxHandle> h;
    bool pending = false;
    int flush_rc = PX_OK;  // a write-behind failure not yet returned to the caller
    std::map<uint32_t, std::unique_ptr<PiXiuChunk>> closed;
};

inline UsedNum::operator uint16_t() const {
    if (owner) owner->sync_pending();
    return n;
}

inline PiXiuStr *PiXiuChunk::getitem(int idx) {
    if (idx < 0) return nullptr;
    if (owner) owner->sync_pending();
    if ((size_t)idx >= cache.size()) cache.resize((size_t)idx + 1);
    std::vector<uint8_t> &c = cache[(size_t)idx];
    if (c.empty()) {
        px_rec r = {0, chunk, (uint32_t)idx, 0, PXSG_MAX_TO};
        std::vector<uint8_t> buf(PXSG_MAX_TO + 8);
        uint64_t off[2] = {0, 0};
        if (px_export(owner->ctx, 1, &r, buf.data(), buf.size(), off) != PX_OK) return nullptr;
        c.resize(2 + off[1]);
        uint16_t len = (uint16_t)off[1];
        memcpy(c.data(), &len, 2);
        memcpy(c.data() + 2, buf.data(), off[1]);
    }
    return reinterpret_cast<PiXiuStr *>(c.data());
}

#endif
