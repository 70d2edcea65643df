// px_kernels.hip — CDNA4 (gfx950) kernels for the PiXiu batch compress/query core.
//
// Execution model: one 64-lane wavefront per independent unit of serial work
// (a shard's suffix tree for setitem, a query's expansion for getitem).  The
// serial state machine lives in wave-uniform (scalar) registers; the 64 lanes are
// used where the work is wide: edge-label fast-forward compares, 16-slot hash
// probes, escape scans, and coalesced byte copies.  See DESIGN.md §3.
//
//   k_doc_len      escape-count pass  -> escaped doc length per record   (PiXiuStr.cpp:228-271)
//   k_doc_write    escape + assemble  -> esc(k)+[251,0](+esc(v)+[251,2]) (PiXiuCtrl.cpp:31-44)
//   k_gst_encode   Ukkonen GST walk + stream encoder, one wave per shard  (SuffixTree.cpp:144-304,
//                                                                           PiXiuStr.cpp:16-118)
//   k_compact      scratch -> packed compressed store
//   k_tokenize     segment index over compressed bytes (token grammar of PiXiuStr.h:139-192)
//   k_decode       PXSGen expansion (compat | exact), one wave per query  (PiXiuStr.h:129-198)
//   k_rehash       child-map migration into a larger table
#include <hip/hip_runtime.h>

#include "px_common.h"

using namespace px;

#define PX_DEV __device__ __forceinline__

namespace {

PX_DEV uint32_t lane_id() { return threadIdx.x & 63u; }

#ifdef PX_TRACE
// debug build only: per-byte encoder message log (cmd, pos, byte) of shard 0
constexpr uint32_t kTraceCap = 1u << 22;
__device__ int32_t g_trace[kTraceCap];
__device__ uint32_t g_trace_n;
#define PX_TRACE_MSG(cmd, pos, val)                                         \
    do {                                                                    \
        if (blockIdx.x == 0 && lane_id() == 0 && g_trace_n + 3 < kTraceCap) { \
            g_trace[g_trace_n] = (int32_t)(cmd);                            \
            g_trace[g_trace_n + 1] = (int32_t)(pos);                        \
            g_trace[g_trace_n + 2] = (int32_t)(val);                        \
            g_trace_n += 3;                                                 \
        }                                                                   \
    } while (0)
#define PX_TRACE_STATE(k)                                                                     \
    do {                                                                                        \
        PX_TRACE_MSG(-100 - (int32_t)(counter + (k)), act_node, act_doc);                       \
        PX_TRACE_MSG(act_direct, act_off + (k), remainder + (int32_t)(k));                      \
        PX_TRACE_MSG(n_nodes, pools, used);                                                     \
    } while (0)
#else
#define PX_TRACE_STATE(k) \
    do {                  \
    } while (0)
#define PX_TRACE_MSG(cmd, pos, val) \
    do {                            \
    } while (0)
#endif
PX_DEV uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
PX_DEV int32_t unii(int32_t v) { return (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)v); }
PX_DEV uint64_t uni64(uint64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}
PX_DEV uint64_t ballot(bool p) { return __ballot(p); }
PX_DEV uint32_t ffs64(uint64_t m) { return (uint32_t)__ffsll((unsigned long long)m) - 1u; }
PX_DEV uint32_t readlane(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
PX_DEV uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

// ====================================================================== escape
// One wave per record (grid-stride).  doc_len = esc(k)+2 (+ esc(v)+2 when vlen>0).
__global__ void __launch_bounds__(256) k_doc_len(uint32_t n, const uint8_t *keys, const uint64_t *koff,
                                                 const uint8_t *vals, const uint64_t *voff,
                                                 uint32_t *doc_len) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        uint64_t ka = koff[r], kb = koff[r + 1], va = voff[r], vb = voff[r + 1];
        uint32_t cnt = 0;
        for (uint64_t p = ka + lane; p < kb; p += 64) cnt += keys[p] == kEsc;
        for (uint64_t p = va + lane; p < vb; p += 64) cnt += vals[p] == kEsc;
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
        if (lane == 0) {
            uint64_t kl = kb - ka, vl = vb - va;
            uint64_t len = kl + 2 + (vl ? vl + 2 : 0) + cnt;
            doc_len[r] = (kl == 0 || len > (uint64_t)kMaxDoc) ? 0xffffffffu : (uint32_t)len;
        }
    }
}

// escape src[a,b) into dst at lane-parallel positions; returns bytes written (uniform)
PX_DEV uint32_t escape_span(const uint8_t *src, uint64_t a, uint64_t b, uint8_t *dst) {
    const uint32_t lane = lane_id();
    uint32_t w = 0;
    for (uint64_t p = a; p < b; p += 64) {
        uint64_t q = p + lane;
        bool live = q < b;
        uint8_t c = live ? src[q] : 0;
        bool e = live && c == kEsc;
        uint64_t em = ballot(e);
        uint32_t before = __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0));
        uint32_t o = w + lane + before;
        if (live) {
            dst[o] = c;
            if (e) dst[o + 1] = kEsc;
        }
        uint32_t nlive = (uint32_t)min((uint64_t)64, b - p);
        w += nlive + (uint32_t)__popcll(em);
    }
    return w;
}

__global__ void __launch_bounds__(256) k_doc_write(uint32_t n, const uint8_t *keys, const uint64_t *koff,
                                                   const uint8_t *vals, const uint64_t *voff,
                                                   uint8_t *const *dst_ptr) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        uint8_t *dst = dst_ptr[r];
        if (dst == nullptr) continue;
        uint64_t ka = koff[r], kb = koff[r + 1], va = voff[r], vb = voff[r + 1];
        uint32_t w = escape_span(keys, ka, kb, dst);
        if (lane == 0) {
            dst[w] = kEsc;
            dst[w + 1] = kKeyEnd;
        }
        w += 2;
        if (vb > va) {
            w += escape_span(vals, va, vb, dst + w);
            if (lane == 0) {
                dst[w] = kEsc;
                dst[w + 1] = kValEnd;
            }
        }
    }
}

// ====================================================================== GST
constexpr uint32_t kObuf = 2048;   // per-wave output staging (LDS)
constexpr uint32_t kFlushAt = kObuf - 64;

PX_DEV uint32_t hslot(uint32_t parent, uint32_t c) {
    uint32_t h = parent * 0x9E3779B1u ^ (c + 1u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h;
}

struct Edge {
    uint32_t id, link, abs, doc, from, to, flags;
};

struct GstWave {
    // shard arena
    const GstShard *sh;
    uint8_t *text;  // live chunk text base
    uint32_t *doc_base;
    uint4 *nodes;
    uint64_t *hash;
    uint32_t *root_kids;
    uint32_t node_cap, hash_mask, doc_cap;
    // persistent counters
    uint32_t n_nodes, n_docs, chunk_seq, epoch, status;
    int32_t pools, used, pool_open;
    uint64_t ctext_off, ub;
    // current doc
    uint32_t cur, cur_base, cur_len;
    // active point (SuffixTree.h:33-40)
    uint32_t act_node, act_doc, act_direct, act_off, counter;
    int32_t remainder;
    // encoder (PiXiuStr.cpp:17-26 statics, per wave here)
    uint32_t out, flushed, run, run_idx, run_to, applied, held, h_c, h_idx, h_pos;
    uint8_t *out_dst;
    uint8_t *obuf;  // LDS

    PX_DEV uint32_t tbyte(uint32_t rel) const { return uni(text[rel]); }

    PX_DEV Edge load(uint32_t id) const {
        uint4 v = nodes[id];
        Edge e;
        e.id = id;
        e.link = uni(v.x);
        e.abs = uni(v.y);
        e.doc = uni(v.z) & 0xffffu;
        e.from = uni(v.z) >> 16;
        e.to = uni(v.w) & 0xffffu;
        e.flags = uni(v.w) >> 16;
        return e;
    }
    PX_DEV void store(const Edge &e) {  // whole node: only for a node just created
        nodes[e.id] = make_uint4(e.link, e.abs, e.doc | (e.from << 16), e.to | (e.flags << 16));
    }
    // label and flags of an existing node.  Never the suffix link: a cached Edge may
    // hold a stale link (set_link on the same node after it was loaded).
    PX_DEV void store_label(const Edge &e) {
        uint32_t *w = reinterpret_cast<uint32_t *>(&nodes[e.id]);
        w[1] = e.abs;
        w[2] = e.doc | (e.from << 16);
        w[3] = e.to | (e.flags << 16);
    }
    PX_DEV void set_link(uint32_t id, uint32_t link) { nodes[id].x = link; }
    PX_DEV uint32_t flags_of(uint32_t id) const { return uni(nodes[id].w) >> 16; }

    PX_DEV void fail(uint32_t code) {
        if (status == kOk) status = code;
    }

    // MemPool::p_malloc block accounting (MemPool.cpp:7-37)
    PX_DEV void charge(int32_t blocks) {
        if (!pool_open) {
            pool_open = 1;
            ++pools;
            used = 0;
        }
        if (blocks > kPoolBlocks - used) {
            ++pools;
            used = 0;
        }
        used += blocks;
    }

    PX_DEV uint32_t doc_len_of(uint32_t d) const { return uni(doc_base[d + 1]) - uni(doc_base[d]); }

    // byte the reference reads through strs[doc]->data[pos]; past the end it reads
    // heap bytes (UB) -> modelled as a value matching nothing, counted.
    PX_DEV int32_t stale_byte(uint32_t doc, uint32_t pos) {
        uint32_t base = uni(doc_base[doc]);
        uint32_t len = uni(doc_base[doc + 1]) - base;
        if (pos >= len) {
            ++ub;
            return -1;
        }
        return (int32_t)tbyte(base + pos);
    }

    // ---- child map: root = direct table, others = 16-wide linear-probe hash ----
    PX_DEV uint32_t child(uint32_t n, uint32_t c, uint32_t *slot_out, bool *found) {
        if (n == kRoot) {
            uint32_t v = uni(root_kids[c]);
            *found = v != kNone;
            *slot_out = c;
            return v;
        }
        const uint32_t lane = lane_id();
        const uint64_t want = ((uint64_t)n << 8) | c;
        uint32_t h = hslot(n, c);
        for (;;) {
            uint32_t s = (h + lane) & hash_mask;
            uint64_t e = lane < kProbe ? hash[s] : 0;
            bool valid = (uint32_t)(e >> 60) == epoch;
            bool match = lane < kProbe && valid && ((e >> 26) & 0x3ffffffffull) == want;
            bool empty = lane < kProbe && !valid;
            uint64_t mm = ballot(match), me = ballot(empty);
            if (mm) {
                uint32_t l = ffs64(mm);
                *found = true;
                *slot_out = (h + l) & hash_mask;
                return uni(readlane((uint32_t)e & ((1u << kNodeBits) - 1u), l));
            }
            if (me) {
                *found = false;
                *slot_out = (h + ffs64(me)) & hash_mask;
                return kNone;
            }
            h += kProbe;
        }
    }
    PX_DEV uint32_t child(uint32_t n, uint32_t c) {
        uint32_t s;
        bool f;
        return child(n, c, &s, &f);
    }
    PX_DEV bool must_child(uint32_t n, uint32_t c, uint32_t *out) {
        uint32_t v = child(n, c);
        if (v == kNone) {
            fail(kErrRefCrash);  // the reference dereferences NULL here
            return false;
        }
        *out = v;
        return true;
    }
    // STNode::set_sub: insert (charges one map entry) or replace an equal key
    PX_DEV void set_child(uint32_t n, uint32_t c, uint32_t kid) {
        uint32_t slot;
        bool found;
        child(n, c, &slot, &found);
        if (!found) charge(kEdgeBlocks);
        if (n == kRoot) {
            root_kids[c] = kid;
        } else {
            hash[slot] = ((uint64_t)epoch << 60) | ((uint64_t)n << 34) | ((uint64_t)c << 26) | kid;
        }
    }

    PX_DEV bool new_node(Edge &e, uint32_t abs, uint32_t doc, uint32_t from, uint32_t to, uint32_t flags) {
        if (n_nodes >= node_cap || n_nodes >= kMaxNodes) {
            fail(kErrCapacity);
            return false;
        }
        charge(kNodeBlocks);
        e.id = n_nodes++;
        e.link = kRoot;
        e.abs = abs;
        e.doc = doc;
        e.from = from;
        e.to = to;
        e.flags = flags;
        store(e);
        return true;
    }

    // ---- fresh chunk (SuffixTree::init_prop, SuffixTree.cpp:61-78) ----
    PX_DEV void clear_tree() {
        const uint32_t lane = lane_id();
        n_nodes = 0;
        pools = 0;
        used = 0;
        pool_open = 0;
        for (uint32_t c = lane; c < 256; c += 64) root_kids[c] = kNone;
        if (++epoch > (uint32_t)kMaxEpoch) {  // epochs exhausted: really clear
            for (uint32_t s = lane; s <= hash_mask; s += 64) hash[s] = 0;
            epoch = 1;
        }
        Edge root;
        new_node(root, 0, 0, 0, 0, 0);
    }

    // ---- stream encoder (PiXiuStr_init_stream) ----
    PX_DEV void flush_obuf(bool all) {
        const uint32_t lane = lane_id();
        uint32_t n = out - flushed;
        if (!all && n < kFlushAt) return;
        __syncthreads();
        for (uint32_t o = lane; o < n; o += 64) out_dst[flushed + o] = obuf[o];
        __syncthreads();
        flushed = out;
    }
    PX_DEV void put(uint32_t b) {
        obuf[out - flushed] = (uint8_t)b;
        ++out;
        flush_obuf(false);
    }
    PX_DEV void flush_run() {
        if (run == 0) return;
        if (run > 6) {
            put(kEsc);
            if (run > 255) {
                uint32_t from = (run_to - run) & 0xffffu;
                put(kBigSign);
                put(run_idx & 0xff);
                put((run_idx >> 8) & 0xff);
                put(run_to & 0xff);
                put((run_to >> 8) & 0xff);
                put(from & 0xff);
                put(from >> 8);
            } else {
                put(run);  // run == 251 aliases the escape (PiXiuStr.cpp:72): kept
                put(run_idx & 0xff);
                put((run_idx >> 8) & 0xff);
                put(run_to & 0xff);
                put((run_to >> 8) & 0xff);
            }
        } else {
            const uint32_t lane = lane_id();
            // the run's bytes were appended literally: they are the doc bytes just consumed
            uint8_t b = lane < run ? text[cur_base + applied - run + lane] : 0;
            if (lane < run) obuf[out - flushed + lane] = b;
            __syncthreads();
            out += run;
            flush_obuf(false);
        }
        run = 0;
    }
    PX_DEV void apply_c(uint32_t idx, uint32_t pos) {
        run_idx = idx;
        run_to = pos + 1;
        ++run;
        ++applied;
    }
    PX_DEV void apply_p() {
        flush_run();
        put(tbyte(cur_base + applied));
        ++applied;
    }
    // one message for doc byte `b` (2-message 251 look-ahead, PiXiuStr.cpp:33-54)
    PX_DEV void feed(bool is_c, uint32_t idx, uint32_t pos, uint32_t b) {
        PX_TRACE_MSG(is_c ? (int32_t)idx : -3, is_c ? pos : 0, b);
        feed_nt(is_c, idx, pos, b);
    }
    PX_DEV void feed_nt(bool is_c, uint32_t idx, uint32_t pos, uint32_t b) {
        if (held) {
            held = 0;
            if (h_c && is_c) {
                apply_c(h_idx, h_pos);
                apply_c(idx, pos);
            } else {
                apply_p();
                apply_p();
            }
        } else if (b == kEsc) {
            held = 1;
            h_c = is_c;
            h_idx = idx;
            h_pos = pos;
        } else if (is_c) {
            apply_c(idx, pos);
        } else {
            apply_p();
        }
    }
    // m (<= 64) consecutive COMPRESS messages (idx, pos0 + k); m251 = bit k set iff byte k is 251
    PX_DEV void feed_bulk(uint32_t idx, uint32_t pos0, uint32_t m, uint64_t m251) {
#ifdef PX_TRACE
        for (uint32_t t = 0; t < m; ++t) PX_TRACE_MSG(idx, pos0 + t, ((m251 >> t) & 1) ? 251 : -1);
#endif
        uint32_t k = 0;
        if (held) {
            feed_nt(true, idx, pos0, (m251 & 1) ? kEsc : 0);
            k = 1;
        }
        if (k >= m) return;
        bool last_held = false;
        if ((m251 >> (m - 1)) & 1) {
            uint64_t span = (m == 64 ? ~0ull : ((1ull << m) - 1)) & ~((1ull << k) - 1);
            uint64_t non = ~m251 & span;  // non-251 bytes in [k, m)
            uint32_t hz = non ? 63u - (uint32_t)__clzll((long long)non) : k - 1;  // highest non-251
            uint32_t L = (m - 1) - hz;  // trailing 251 run length
            last_held = (L & 1) != 0;
        }
        uint32_t cnt = m - k - (last_held ? 1 : 0);
        if (cnt) {
            run += cnt;
            run_idx = idx;
            run_to = pos0 + k + cnt;
            applied += cnt;
        }
        if (last_held) {
            held = 1;
            h_c = 1;
            h_idx = idx;
            h_pos = pos0 + m - 1;
        }
    }

    // ---- Ukkonen step pieces (SuffixTree.cpp:144-289) ----
    PX_DEV void at_root(uint32_t c, bool send) {
        uint32_t e = uni(root_kids[c]);
        if (e == kNone) {
            Edge leaf;
            if (!new_node(leaf, cur_base + counter, cur, counter, cur_len, 0)) return;
            set_child(kRoot, c, leaf.id);
            --remainder;
            if (send) feed(false, 0, 0, c);
        } else {
            Edge ed = load(e);
            act_doc = ed.doc;
            act_direct = ed.from;
            act_off = (act_off + 1) & 0xffffu;
            if (send) feed(true, ed.doc, ed.from, c);
        }
    }

    // overflow_fix: canonise the active point along the current text
    PX_DEV bool canonise(Edge &e) {
        int32_t end = (int32_t)counter;
        int32_t begin = end - (int32_t)act_off;
        uint32_t id;
        if (!must_child(act_node, tbyte(cur_base + counter - act_off), &id)) return false;
        e = load(id);
        int32_t supply;
        while (end - begin > (supply = (int32_t)e.to - (int32_t)e.from)) {
            act_node = e.id;
            begin += supply;
            act_off = (act_off - (uint32_t)supply) & 0xffffu;
            if (!must_child(act_node, tbyte(cur_base + (uint32_t)begin), &id)) return false;
            e = load(id);
            act_direct = e.from;
        }
        return true;
    }

    // split_grow
    PX_DEV bool grow(Edge &e, uint32_t &last_inner) {
        Edge leaf;
        if (!new_node(leaf, cur_base + counter, cur, counter, cur_len, 0)) return false;
        --remainder;
        bool e_leaf = e.id != kRoot && !(e.flags & kFlagKids);
        if ((e_leaf || e.to - e.from > 1) && e.from + act_off != e.to) {
            Edge in;
            if (!new_node(in, e.abs, e.doc, e.from, (e.from + act_off) & 0xffffu, kFlagKids)) return false;
            if (last_inner != kNone) set_link(last_inner, in.id);
            last_inner = in.id;
            set_child(act_node, tbyte(in.abs), in.id);  // replaces e under its first byte
            e.from = in.to;
            e.abs += act_off;
            store_label(e);
            set_child(in.id, tbyte(e.abs), e.id);
            set_child(in.id, tbyte(leaf.abs), leaf.id);
        } else {
            if (last_inner != kNone) set_link(last_inner, e.id);
            last_inner = e.id;
            set_child(e.id, tbyte(leaf.abs), leaf.id);
            if (!(e.flags & kFlagKids)) {
                e.flags |= kFlagKids;
                store_label(e);
            }
        }
        return true;
    }

    // compare the current text from doc position i against the active edge's label
    // (read through the stale active doc, SuffixTree.cpp:171,184) and apply the
    // matching prefix as COMPRESS messages in bulk.  Returns matched length.
    PX_DEV uint32_t fast_forward(const Edge &e, uint32_t i) {
        const uint32_t lane = lane_id();
        uint32_t base_a = uni(doc_base[act_doc]);
        uint32_t len_a = uni(doc_base[act_doc + 1]) - base_a;
        uint32_t limit = min(e.to - e.from - act_off, cur_len - i);
        uint32_t m = 0;
        while (m < limit) {
            uint32_t w = min(64u, limit - m);
            uint32_t t = e.from + act_off + m + lane;  // position in the active doc
            bool live = lane < w;
            uint32_t a = live ? text[cur_base + i + m + lane] : 0;
            bool oob = live && t >= len_a;
            uint32_t b = (live && !oob) ? text[base_a + t] : 0x100u;
            uint64_t mism = ballot(live && (oob || a != b));
            uint64_t m251 = ballot(live && a == kEsc);
            uint32_t got = mism ? ffs64(mism) : w;
            if (got) feed_bulk(e.doc, e.from + act_off + m, got, m251);
            m += got;
            if (mism) {
                if ((mism >> got) & 1ull && readlane((uint32_t)oob, got)) ++ub;
                break;
            }
        }
        return m;
    }

    // SuffixTree::setitem for one doc of `len` bytes already in the arena
    PX_DEV void encode_doc(uint32_t len) {
        cur_len = len;
        remainder = 0;
        counter = 0;
        act_node = kRoot;
        act_doc = act_direct = act_off = 0;
        out = flushed = run = applied = held = 0;
        bool have_e = false;
        Edge e;
        uint32_t i = 0;
        while (i < len && status == kOk) {
            const uint32_t c = tbyte(cur_base + i);
            PX_TRACE_STATE(0);
            if (act_node == kRoot && act_off == 0) {
                ++remainder;
                at_root(c, true);
                ++counter;
                ++i;
                have_e = false;
                continue;
            }
            if (!have_e) {
                int32_t key = stale_byte(act_doc, act_direct);
                uint32_t id;
                if (key < 0) {
                    fail(kErrRefCrash);  // get_sub(garbage) -> NULL deref in the reference
                    break;
                }
                if (!must_child(act_node, (uint32_t)key, &id)) break;
                e = load(id);
                have_e = true;
            }
            if (e.from + act_off == e.to) {
                uint32_t nx = (e.flags & kFlagKids) ? child(e.id, c) : kNone;
                if (nx != kNone) {
                    ++remainder;
                    Edge n = load(nx);
                    act_node = e.id;
                    act_doc = n.doc;
                    act_direct = n.from;
                    act_off = 1;
                    feed(true, n.doc, n.from, c);
                    e = n;  // child(act_node, text[act_doc][act_direct]) == n
                    ++counter;
                    ++i;
                    continue;
                }
            } else if (e.from + act_off < e.to) {
                uint32_t m = fast_forward(e, i);
#ifdef PX_TRACE
                for (uint32_t k = 1; k < m; ++k) PX_TRACE_STATE(k);
#endif
                if (m) {
                    remainder += (int32_t)m;
                    act_off = (act_off + m) & 0xffffu;
                    counter += m;
                    i += m;
                    continue;
                }
            }
            // mismatch: emit PASS, then split/grow along suffix links
            ++remainder;
            feed(false, 0, 0, c);
            uint32_t last_inner = kNone;
            while (remainder > 0 && status == kOk) {
                if (!grow(e, last_inner)) break;
                if (act_node == kRoot || !(flags_of(act_node) & kFlagKids)) {
                    act_off = (act_off - 1) & 0xffffu;
                    act_direct = (act_direct + 1) & 0xffffu;
                    if (act_off > 0) {
                        if (!canonise(e)) break;
                    } else {
                        at_root(c, false);
                        break;
                    }
                } else {
                    act_node = load(act_node).link;
                    if (!canonise(e)) break;
                }
                if (e.from + act_off == e.to) {
                    uint32_t nx = (e.flags & kFlagKids) ? child(e.id, c) : kNone;
                    if (nx != kNone) {
                        Edge n = load(nx);
                        act_node = e.id;
                        act_doc = n.doc;
                        act_direct = n.from;
                        act_off = 1;
                        if (last_inner != kNone) set_link(last_inner, act_node);
                        break;
                    }
                } else if (e.from + act_off < e.to && c == tbyte(e.abs + act_off)) {
                    act_off = (act_off + 1) & 0xffffu;
                    break;
                }
            }
            have_e = false;
            ++counter;
            ++i;
        }
        if (status == kOk) {
            if (held) fail(kErrCorrupt);  // stream ended inside a 251 pair
            flush_run();
            flush_obuf(true);
        }
    }
};

__global__ void __launch_bounds__(64) k_gst_encode(const GstShard *shards, uint32_t n_shards,
                                                   const uint32_t *doc_len, uint8_t *const *comp_dst,
                                                   uint32_t *comp_len, uint32_t *rec_chunk,
                                                   uint32_t *rec_idx, uint32_t *rec_status) {
    __shared__ uint8_t obuf[kObuf];
    const uint32_t s = blockIdx.x;
    if (s >= n_shards) return;
    const GstShard sh = shards[s];
    ShardState st = *sh.st;
    GstWave g;
    g.sh = &shards[s];
    g.doc_base = sh.doc_base;
    g.nodes = sh.nodes;
    g.hash = sh.hash;
    g.root_kids = sh.root_kids;
    g.node_cap = sh.node_cap;
    g.hash_mask = sh.hash_mask;
    g.doc_cap = sh.doc_cap;
    g.n_nodes = uni(st.n_nodes);
    g.n_docs = uni(st.n_docs);
    g.chunk_seq = uni(st.chunk_seq);
    g.epoch = uni(st.epoch);
    g.status = uni(st.status);
    g.pools = unii(st.pools);
    g.used = unii(st.used_blocks);
    g.pool_open = unii(st.pool_open);
    g.ctext_off = uni64(st.ctext_off);
    g.ub = uni64(st.ub_reads);
    g.text = sh.text + g.ctext_off;
    g.obuf = obuf;
    if (g.epoch == 0) {  // brand-new shard
        g.epoch = 0;
        g.clear_tree();
        g.doc_base[0] = 0;
        g.n_docs = 0;
    }
    for (uint32_t r = sh.r0; r < sh.r1; ++r) {
        const uint32_t len = uni(doc_len[r]);
        if (g.status != kOk || len == 0xffffffffu) {
            if (lane_id() == 0) {
                rec_status[r] = g.status != kOk ? g.status : (uint32_t)kErrInval;
                comp_len[r] = 0;
            }
            continue;
        }
        // rotation (PiXiuCtrl.cpp:13-25): before the doc, by pool count or slot count
        if (g.pools >= kRotatePools || g.n_docs == (uint32_t)kChunkSlots) {
            uint32_t shift = uni(g.doc_base[g.n_docs]);
            g.ctext_off += shift;
            g.text = sh.text + g.ctext_off;
            g.n_docs = 0;
            g.doc_base[0] = 0;
            ++g.chunk_seq;
            g.clear_tree();
        }
        if (g.n_docs >= g.doc_cap) {
            g.fail(kErrCapacity);
            if (lane_id() == 0) rec_status[r] = g.status;
            continue;
        }
        g.cur = g.n_docs;
        g.cur_base = uni(g.doc_base[g.cur]);
        g.doc_base[g.cur + 1] = g.cur_base + len;
        g.out_dst = comp_dst[r];
        g.encode_doc(len);
        ++g.n_docs;
        if (lane_id() == 0) {
            comp_len[r] = g.out;
            rec_chunk[r] = g.chunk_seq;
            rec_idx[r] = g.cur;
            rec_status[r] = g.status;
        }
    }
    if (lane_id() == 0) {
        ShardState o;
        o.n_nodes = g.n_nodes;
        o.pools = g.pools;
        o.used_blocks = g.used;
        o.pool_open = g.pool_open;
        o.n_docs = g.n_docs;
        o.chunk_seq = g.chunk_seq;
        o.epoch = g.epoch;
        o.status = g.status;
        o.ctext_off = g.ctext_off;
        o.ub_reads = g.ub;
        *sh.st = o;
    }
}

// ====================================================================== store
// Copy each record's compressed bytes from scratch into the packed store.
__global__ void __launch_bounds__(256) k_compact(uint32_t n, uint8_t *const *src, const uint32_t *len,
                                                 uint8_t *dst, const uint64_t *dst_off) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        const uint8_t *s = src[r];
        uint8_t *d = dst + dst_off[r];
        uint32_t l = len[r];
        for (uint32_t o = lane; o < l; o += 64) d[o] = s[o];
    }
}

// Segment index over the token grammar of PXSGen (PiXiuStr.h:139-192):
// entries (src_start, comp_start | kind << 30) + a sentinel (src_total, comp_len).
// kind 0 plain (literals and 251-pairs, copied verbatim), 2 record, 1 skip (251 + 3..6).
constexpr uint32_t kSegRecord = 2u << 30, kSegSkip = 1u << 30, kSegMask = (1u << 30) - 1;

__global__ void __launch_bounds__(256) k_tokenize(uint32_t n, const RecSlot *slots_in, uint2 *const *seg_out,
                                                  uint32_t *nseg_out, uint32_t *status) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        const uint8_t *comp = slots_in[r].comp;
        const uint32_t len = slots_in[r].comp_len;
        uint2 *seg = seg_out[r];
        uint32_t ns = 0, p = 0, wb = 0, err = 0, plain_start = 0;
        int32_t src = 0;
        bool plain_open = false;
        uint32_t b = lane < len ? comp[lane] : 0;
        while (p < len) {
            if (p >= wb + 64 || (p + 8 > wb + 64 && wb + 64 < len)) {
                wb = p;
                b = wb + lane < len ? comp[wb + lane] : 0;
            }
            if (!plain_open) {
                if (lane == 0) seg[ns] = make_uint2((uint32_t)src, p);
                ++ns;
                plain_open = true;
                plain_start = p;
            }
            uint32_t lim = min(64u, len - wb);
            uint64_t m = ballot(lane >= p - wb && lane < lim && b == kEsc);
            if (!m) {
                uint32_t adv = wb + lim - p;
                p += adv;
                src += (int32_t)adv;
                continue;
            }
            uint32_t q = wb + ffs64(m);
            src += (int32_t)(q - p);
            p = q;
            if (p + 8 > wb + 64 && wb + 64 < len) continue;  // refill so the token is in the window
            if (p + 1 >= len) {
                err = kErrCorrupt;
                break;
            }
            uint32_t nx = readlane(b, p + 1 - wb);
            if (nx == kKeyEnd || nx == kEsc || nx == kValEnd) {
                p += 2;
                src += 2;
                continue;
            }
            // record or skip token: closes the plain segment (dropped if empty)
            if (plain_start == p) --ns;
            if (nx == kBigSign || nx > 6) {
                uint32_t size = nx == kBigSign ? 8u : 6u;
                if (p + size > len) {
                    err = kErrCorrupt;
                    break;
                }
                uint32_t to = readlane(b, p + 4 - wb) | (readlane(b, p + 5 - wb) << 8);
                uint32_t from = nx == kBigSign ? (readlane(b, p + 6 - wb) | (readlane(b, p + 7 - wb) << 8))
                                               : ((to - nx) & 0xffffu);
                if (lane == 0) seg[ns] = make_uint2((uint32_t)src, p | kSegRecord);
                ++ns;
                src += (int32_t)to - (int32_t)from;
                p += size;
            } else {
                if (lane == 0) seg[ns] = make_uint2((uint32_t)src, p | kSegSkip);
                ++ns;
                p += 1;
            }
            plain_open = false;
        }
        if (!err) {
            if (plain_open && plain_start == len) --ns;
            if (lane == 0) seg[ns] = make_uint2((uint32_t)src, len);
        }
        if (lane == 0) {
            nseg_out[r] = err ? 0 : ns;
            status[r] = err;
        }
    }
}

// ====================================================================== decode
PX_DEV void wave_copy(uint8_t *dst, const uint8_t *src, uint32_t n) {
    for (uint32_t o = lane_id(); o < n; o += 64) dst[o] = src[o];
}

// first segment whose end is beyond `from` (64-ary search)
PX_DEV uint32_t seg_search(const uint2 *seg, uint32_t nseg, int32_t from) {
    const uint32_t lane = lane_id();
    uint32_t lo = 0, hi = nseg;  // answer in [lo, hi]; seg[k+1].x > from
    while (hi - lo > 64) {
        uint32_t step = (hi - lo + 63) / 64;
        uint32_t k = lo + lane * step;
        bool le = k < hi && (int32_t)seg[k + 1].x <= from;  // segment k ends at or before from
        uint64_t m = ballot(le);
        uint32_t cnt = (uint32_t)__popcll(m);  // prefix of lanes with le (monotone)
        uint32_t nlo = cnt ? lo + (cnt - 1) * step + 1 : lo;
        uint32_t nhi = min(hi, lo + cnt * step);
        lo = uni(nlo);
        hi = uni(nhi);
    }
    uint32_t k = lo + lane;
    bool le = k < hi && (int32_t)seg[k + 1].x <= from;
    return uni(lo + (uint32_t)__popcll(ballot(le)));
}

__global__ void __launch_bounds__(64) k_decode(const DecodeQuery *qs, uint32_t nq, const RecSlot *const *chunk_slots,
                                               uint8_t *out, uint32_t *out_len, uint32_t *status,
                                               Frame *scratch, uint32_t depth_cap) {
    const uint32_t lane = lane_id();
    Frame *stk = scratch + (size_t)blockIdx.x * depth_cap;
    for (uint32_t qi = blockIdx.x; qi < nq; qi += gridDim.x) {
        const DecodeQuery q = qs[qi];
        const RecSlot *slots = uni(q.chunk) == kNone ? nullptr : chunk_slots[uni(q.chunk)];
        const bool compat = uni(q.mode) == 0;
        uint8_t *o = out + uni64(q.out_off);
        const uint32_t qcap = uni(q.out_cap);
        uint32_t outp = 0, err = 0, depth = 0;
        bool capped = false;

        // push helper (inline): frame for record `r`, range [from, to), cap
        auto push = [&](uint32_t r, int32_t from, int32_t to, uint32_t cap) -> bool {
            if (depth >= depth_cap) {
                err = kErrDepth;
                return false;
            }
            const RecSlot sl = slots[r];
            uint32_t nseg = uni(sl.nseg);
            Frame f;
            f.rec = r;
            f.from = from;
            f.len = to - from;
            f.ret = 0;
            f.seg = nseg ? seg_search(sl.seg, nseg, from) : 0;
            f.src = f.seg < nseg ? unii((int32_t)sl.seg[f.seg].x) : 0;
            f.cap = cap;
            f.state = 0;
            f.pstart = 0;
            f.sub_from = f.sub_to = f.supply = 0;
            stk[depth] = f;
            ++depth;
            return true;
        };

        if (uni(q.chunk) == kNone || !push(uni(q.idx), unii(q.from), unii(q.to), qcap)) {
            if (lane == 0) {
                out_len[qi] = 0;
                status[qi] = err ? err : kErrInval;
            }
            continue;
        }
        while (depth > 0 && !err) {
            __builtin_amdgcn_wave_barrier();
            Frame f = stk[depth - 1];
            f.rec = uni(f.rec);
            f.from = unii(f.from);
            f.len = unii(f.len);
            f.ret = unii(f.ret);
            f.src = unii(f.src);
            f.seg = uni(f.seg);
            f.cap = uni(f.cap);
            f.state = uni(f.state);
            f.pstart = uni(f.pstart);
            f.sub_from = unii(f.sub_from);
            f.sub_to = unii(f.sub_to);
            f.supply = unii(f.supply);
            const RecSlot sl = slots[f.rec];
            const uint8_t *comp = sl.comp;
            const uint2 *seg = sl.seg;
            const uint32_t nseg = uni(sl.nseg);
            bool pop = false;

            if (f.state != 0) {  // a child just returned
                if (outp >= f.cap) {
                    pop = true;
                } else {
                    if (f.state == 2) {  // periodic: repeat the child's output to n bytes
                        uint32_t produced = outp - f.pstart;
                        uint32_t n = (uint32_t)(f.sub_to - f.sub_from);
                        if (produced == 0) {
                            err = kErrHang;
                            break;
                        }
                        if (produced < n) {
                            uint32_t end = min(f.pstart + n, f.cap);
                            __threadfence_block();
                            for (uint32_t k = produced + lane; f.pstart + k < end; k += 64)
                                o[f.pstart + k] = o[f.pstart + (k % produced)];
                            outp = end;
                            if (outp >= f.cap) pop = true;
                        }
                    }
                    if (!pop) {
                        f.ret += f.sub_to - f.sub_from;
                        f.src += f.supply;
                        ++f.seg;
                        f.state = 0;
                    }
                }
            }
            bool pushed = false;
            while (!pop && !pushed && f.ret < f.len && f.seg < nseg) {
                const uint32_t sx = uni(seg[f.seg].x), sy = uni(seg[f.seg].y);
                const uint32_t cs = sy & kSegMask;
                if (sy & kSegRecord) {
                    const uint8_t *t = comp + cs;
                    uint32_t sign = uni(t[1]);
                    int32_t ridx = (int32_t)uni(rd16(t + 2));
                    int32_t rto = (int32_t)uni(rd16(t + 4));
                    int32_t rfrom = sign == kBigSign ? (int32_t)uni(rd16(t + 6)) : ((rto - (int32_t)sign) & 0xffff);
                    int32_t supply = rto - rfrom;
                    if (f.src - 1 + supply >= f.from) {
                        int32_t sub_from = rfrom + max(0, f.from - f.src);
                        int32_t sub_to = min(rto, sub_from + (f.len - f.ret));
                        int32_t stop = compat ? f.ret : max(f.src, f.from);
                        bool periodic = sub_from < stop && stop < sub_to && (uint32_t)ridx == f.rec;
                        f.state = periodic ? 2 : 1;
                        f.pstart = outp;
                        f.sub_from = sub_from;
                        f.sub_to = sub_to;
                        f.supply = supply;
                        __builtin_amdgcn_wave_barrier();
                        stk[depth - 1] = f;
                        uint32_t ccap = periodic ? min(f.cap, outp + (uint32_t)(sub_to - sub_from)) : f.cap;
                        bool ok = periodic ? push(f.rec, sub_from, stop, ccap) : push((uint32_t)ridx, sub_from, sub_to, ccap);
                        if (!ok) break;
                        pushed = true;
                        break;
                    }
                    f.src += supply;
                    ++f.seg;
                } else if (sy & kSegSkip) {
                    ++f.seg;
                } else {
                    const int32_t e = (int32_t)uni(seg[f.seg + 1].x);
                    const int32_t p0 = max((int32_t)sx, f.from);
                    if (p0 < e) {
                        uint32_t avail = (uint32_t)(e - p0);
                        uint32_t need = (uint32_t)(f.len - f.ret);
                        uint32_t nb = min(avail, need);
                        if (avail > need && compat) {
                            // the range ends here: if the last byte opens a 251 pair, the pair
                            // is written whole (per-token length check, PiXiuStr.h:136,142-147)
                            uint32_t ci = cs + (uint32_t)(p0 - (int32_t)sx) + nb - 1;
                            uint32_t run = 0;
                            for (;;) {
                                uint32_t lo = ci + 1 - run;  // scan [lo-64, lo)
                                uint32_t span = min(64u, lo - cs);
                                bool is_e = lane < span && comp[lo - 1 - lane] == kEsc;
                                uint64_t nm = ballot(lane < span && !is_e);
                                if (nm) {
                                    run += ffs64(nm);
                                    break;
                                }
                                run += span;
                                if (span < 64) break;
                            }
                            if (run & 1) nb += 1;
                        }
                        uint32_t room = f.cap > outp ? f.cap - outp : 0;
                        uint32_t w = min(nb, room);
                        wave_copy(o + outp, comp + cs + (uint32_t)(p0 - (int32_t)sx), w);
                        outp += w;
                        f.ret += (int32_t)nb;
                        if (w < nb || outp >= f.cap) {
                            pop = true;
                            break;
                        }
                    }
                    f.src = e;
                    ++f.seg;
                }
            }
            if (err) break;
            if (pushed) continue;
            // frame finished (or stopped by its consumer)
            --depth;
            if (depth == 0 && outp >= qcap && pop) capped = true;
        }
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            out_len[qi] = outp;
            status[qi] = err ? err : (capped ? (uint32_t)kErrSpace : (uint32_t)kOk);
        }
    }
}

// ====================================================================== migrate
__global__ void __launch_bounds__(256) k_rehash(const uint64_t *old_tab, uint32_t old_cap, uint32_t epoch,
                                                uint64_t *new_tab, uint32_t new_mask) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= old_cap) return;
    uint64_t e = old_tab[i];
    if ((uint32_t)(e >> 60) != epoch) return;
    uint32_t parent = (uint32_t)(e >> 34) & ((1u << kNodeBits) - 1u);
    uint32_t c = (uint32_t)(e >> 26) & 0xffu;
    uint32_t h = hslot(parent, c);
    for (;;) {
        uint32_t s = h & new_mask;
        unsigned long long prev = atomicCAS((unsigned long long *)&new_tab[s], 0ull, (unsigned long long)e);
        if (prev == 0ull) return;
        ++h;
    }
}

}  // namespace

// ---------------------------------------------------------------------- launchers
namespace px {

hipError_t launch_doc_len(hipStream_t s, uint32_t n, const uint8_t *keys, const uint64_t *koff,
                          const uint8_t *vals, const uint64_t *voff, uint32_t *doc_len) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_doc_len<<<blocks, 256, 0, s>>>(n, keys, koff, vals, voff, doc_len);
    return hipGetLastError();
}

hipError_t launch_doc_write(hipStream_t s, uint32_t n, const uint8_t *keys, const uint64_t *koff,
                            const uint8_t *vals, const uint64_t *voff, uint8_t *const *dst) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_doc_write<<<blocks, 256, 0, s>>>(n, keys, koff, vals, voff, dst);
    return hipGetLastError();
}

hipError_t launch_gst_encode(hipStream_t s, const GstShard *shards, uint32_t n_shards, const uint32_t *doc_len,
                             uint8_t *const *comp_dst, uint32_t *comp_len, uint32_t *rec_chunk,
                             uint32_t *rec_idx, uint32_t *rec_status) {
    if (!n_shards) return hipSuccess;
    k_gst_encode<<<n_shards, 64, 0, s>>>(shards, n_shards, doc_len, comp_dst, comp_len, rec_chunk, rec_idx,
                                         rec_status);
    return hipGetLastError();
}

hipError_t launch_compact(hipStream_t s, uint32_t n, uint8_t *const *src, const uint32_t *len, uint8_t *dst,
                          const uint64_t *dst_off) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_compact<<<blocks, 256, 0, s>>>(n, src, len, dst, dst_off);
    return hipGetLastError();
}

hipError_t launch_tokenize(hipStream_t s, uint32_t n, const RecSlot *slots, uint2 *const *seg_out,
                           uint32_t *nseg_out, uint32_t *status) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_tokenize<<<blocks, 256, 0, s>>>(n, slots, seg_out, nseg_out, status);
    return hipGetLastError();
}

hipError_t launch_decode(hipStream_t s, const DecodeQuery *qs, uint32_t nq, const RecSlot *const *chunk_slots,
                         uint8_t *out, uint32_t *out_len, uint32_t *status, Frame *scratch, uint32_t depth_cap,
                         uint32_t n_waves) {
    if (!nq) return hipSuccess;
    k_decode<<<n_waves, 64, 0, s>>>(qs, nq, chunk_slots, out, out_len, status, scratch, depth_cap);
    return hipGetLastError();
}

int debug_trace_take(int32_t *out, uint32_t cap) {
#ifdef PX_TRACE
    uint32_t n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_trace_n), 4) != hipSuccess) return -1;
    n = n < cap ? n : cap;
    if (n && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), (size_t)n * 4) != hipSuccess) return -1;
    uint32_t z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_trace_n), &z, 4);
    return (int)(n / 3);
#else
    (void)out;
    (void)cap;
    return -1;
#endif
}

hipError_t launch_rehash(hipStream_t s, const uint64_t *old_tab, uint32_t old_cap, uint32_t epoch,
                         uint64_t *new_tab, uint32_t new_mask) {
    if (!old_cap) return hipSuccess;
    k_rehash<<<(old_cap + 255) / 256, 256, 0, s>>>(old_tab, old_cap, epoch, new_tab, new_mask);
    return hipGetLastError();
}

}  // namespace px
