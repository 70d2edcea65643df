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
//   k_decode_keys  the same body for stored-key prefixes (setitem's CritBit inserts, prefix iter)
//   k_rehash       child-map migration into a larger table
#include <hip/hip_runtime.h>

#include "px_common.h"

using namespace px;

#define PX_DEV __device__ __forceinline__
// explicit address spaces: pointers reached through structs would otherwise be
// flat, and every flat access waits for all outstanding vector-memory AND LDS ops
#define PX_GAS __attribute__((address_space(1)))
#define PX_LAS __attribute__((address_space(3)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

PX_DEV uint32_t lane_id() { return threadIdx.x & 63u; }
PX_DEV u32x4 mk4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return u32x4{a, b, c, d}; }

#ifdef PX_TRACE
// debug build only: per-byte encoder message log (cmd, pos, byte) of shard 0
constexpr uint32_t kTraceCap = 1u << 22;
__device__ int32_t g_trace[kTraceCap];
__device__ uint32_t g_trace_n;
#define PX_TRACE_MSG(cmd, pos, val)                                         \
    do {                                                                    \
        if (blockIdx.x == 0 && threadIdx.x == 0 && g_trace_n + 3 < kTraceCap) { \
            g_trace[g_trace_n] = (int32_t)(cmd);                            \
            g_trace[g_trace_n + 1] = (int32_t)(pos);                        \
            g_trace[g_trace_n + 2] = (int32_t)(val);                        \
            g_trace_n += 3;                                                 \
        }                                                                   \
    } while (0)
#define PX_TRACE_STATE(k)                                                                     \
    do {                                                                                        \
        PX_TRACE_MSG(-100 - (int32_t)(i + (k)), act_node, act_doc);                       \
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
// a value the compiler must keep in a VGPR (it cannot prove it wave-uniform)
PX_DEV uint32_t vreg(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}
PX_DEV uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

// inclusive wave prefix sum on DPP row shifts and row broadcasts (no LDS round trips)
PX_DEV int32_t wave_incl_scan_dpp(int32_t x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 into rows 2, 3
    return x;
}

#ifdef PX_PROFILE
// debug build only: per-category counters and shader-clock cycles of k_gst_encode
enum { P_BYTES, P_FF_CALLS, P_FF_BYTES, P_PASS, P_ITERS, P_LOOKUPS, P_PROBES, P_ROOT, P_WALK, P_LINK, P_CANON_LVL,
       P_T_TOTAL, P_T_FF, P_T_DERIVE, P_T_WALK, P_T_SPLIT, P_T_GROW, P_T_CANON, P_T_END, P_T_ROOT, P_T_ENC,
       P_KEYMISS, P_T_KEY, P_T_LOOK,
       P_D_BATCH, P_D_LANEIT, P_D_SERIAL, P_D_COMMIT, P_D_FLAGGED, P_D_SHORT, P_D_PUSH, P_D_T_TOTAL, P_D_T_LANE,
       P_G_NOSPLIT, P_G_T_LEAF, P_G_T_SPLIT, P_G_T_ADD,
       P_E_LOOK, P_E_OFF1, P_E_OFF2, P_E_OFF3, P_E_OFF4P, P_K_CACHED, P_K_LOAD1, P_K_LOADN,
       P_DF_NONE, P_DF_TOPREF, P_DF_CAP, P_DF_NOLINK, P_DF_OVER, P_DF_LPER, P_DF_DEPTH, P_DF_RANGE, P_DF_BADREC,
       P_D_TOPB, P_D_SUBB, P_D_TOPC, P_D_MAXIT, P_D_T_ASSIGN, P_D_ROUNDS, P_D_SPILL, P_N };
__device__ unsigned long long g_prof[P_N];
#define PX_CNT(k, v) (prof[k] += (v))
#define PX_T0() uint64_t _t0 = __builtin_amdgcn_s_memtime()
#define PX_T1(k) (prof[k] += __builtin_amdgcn_s_memtime() - _t0)
#define PX_FR(r) (freason = freason ? freason : (r))
#else
#define PX_FR(r) ((void)0)
#define PX_CNT(k, v) ((void)0)
#define PX_T0() ((void)0)
#define PX_T1(k) ((void)0)
#endif

// ====================================================================== escape
// One wave per record (grid-stride).  doc_len = esc(k)+2 (+ esc(v)+2 when vlen>0).
// It also defines every per-record result word of the batch (status OK / EINVAL,
// comp_len, chunk and slot all-ones) so no value can survive from an earlier batch
// that used the same scratch: each later kernel overwrites them, never relies on them.
__global__ void __launch_bounds__(256) k_doc_len(uint32_t n, const uint8_t *keys, const uint64_t *koff,
                                                 const uint8_t *vals, const uint64_t *voff,
                                                 uint32_t *doc_len, uint32_t *rec_init) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        if (!vals) {  // ready docs (reinsert, PiXiuCtrl.cpp:39-40): taken as they are
            if (lane == 0) {
                const uint64_t len = koff[r + 1] - koff[r];
                const bool bad = len == 0 || len > (uint64_t)kMaxDoc;
                doc_len[r] = bad ? 0xffffffffu : (uint32_t)len;
                if (rec_init) {
                    rec_init[r] = rec_init[n + r] = rec_init[2 * n + r] = 0xffffffffu;
                    rec_init[3 * n + r] = bad ? (uint32_t)kErrInval : (uint32_t)kOk;
                }
            }
            continue;
        }
        uint64_t ka = koff[r], kb = koff[r + 1], va = voff[r], vb = voff[r + 1];
        uint32_t cnt = 0;
        for (uint64_t p = ka + lane; p < kb; p += 64) cnt += keys[p] == kEsc;
        for (uint64_t p = va + lane; p < vb; p += 64) cnt += vals[p] == kEsc;
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
        if (lane == 0) {
            uint64_t kl = kb - ka, vl = vb - va;
            uint64_t len = kl + 2 + (vl ? vl + 2 : 0) + cnt;
            const bool bad = kl == 0 || len > (uint64_t)kMaxDoc;
            doc_len[r] = bad ? 0xffffffffu : (uint32_t)len;
            if (rec_init) {  // [comp_len | chunk | idx | status] x n, after doc_len
                rec_init[r] = 0xffffffffu;
                rec_init[n + r] = 0xffffffffu;
                rec_init[2 * n + r] = 0xffffffffu;
                rec_init[3 * n + r] = bad ? (uint32_t)kErrInval : (uint32_t)kOk;
            }
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
        if (!vals) {  // a ready doc: copied verbatim
            for (uint64_t p = koff[r] + lane; p < koff[r + 1]; p += 64) dst[p - koff[r]] = keys[p];
            continue;
        }
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
// One wave per shard.  The serial Ukkonen walk (SuffixTree.cpp:144-289) and the
// stream encoder (PiXiuStr.cpp:16-118) run on wave-uniform values; the lanes are
// used for wide work: 64-byte edge-label fast-forward compares, 4-entry bucket
// probes (one 64-byte line per probe), the current doc's 256-byte byte window,
// and the encoder's output staging.  Per shard, LDS holds the root's 256 child
// entries, the first 256 doc starts and the output staging buffer.
constexpr uint32_t kPassMsg = 0xffffffffu;  // NO_COMPRESS (a COMPRESS idx is at most 65,534)
constexpr uint32_t kDocCache = 256;  // doc starts cached in LDS
constexpr uint32_t kRootSlot = 0x80000000u;
constexpr uint32_t kWin = 256;  // current-doc window (4 bytes per lane)

// GST blocks are exactly one wave: LDS ops of a wave execute in order, so lanes
// exchanging data through LDS need only a compiler barrier, not s_barrier (whose
// fence would also wait for every outstanding global load and store)
PX_DEV void wave_sync() { asm volatile("" ::: "memory"); }

PX_DEV uint32_t hslot(uint32_t parent, uint32_t c) {
    uint32_t h = parent * 0x9E3779B1u ^ (c + 1u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h;
}

// an edge = the child's entry in its parent's map.  cnt = the child's own child
// count, saturated at 3; slot = where the entry lives (root table, one of the
// parent's two inline slots, or a hash slot).
// Kept in its packed entry form (the three words a map entry stores), so loads and
// stores move it without repacking and it occupies four scalar registers, not seven.
struct Edge {
    uint32_t w0;    // child id | child count (saturated at 3) << 26
    uint32_t w1;    // label doc | from << 16
    uint32_t w2;    // label to | key (first byte) << 16
    uint32_t slot;
    PX_DEV uint32_t id() const { return w0 & kNodeMask; }
    PX_DEV uint32_t cnt() const { return (w0 >> 26) & 3u; }
    PX_DEV uint32_t doc() const { return w1 & 0xffffu; }
    PX_DEV uint32_t from() const { return w1 >> 16; }
    PX_DEV uint32_t to() const { return w2 & 0xffffu; }
    PX_DEV uint32_t key() const { return (w2 >> 16) & 0xffu; }
    PX_DEV void set(uint32_t id, uint32_t cnt, uint32_t doc, uint32_t from, uint32_t to, uint32_t key) {
        w0 = id | cnt << 26;
        w1 = doc | from << 16;
        w2 = to | key << 16;
    }
    PX_DEV void set_from(uint32_t f) { w1 = (w1 & 0xffffu) | f << 16; }
    PX_DEV void set_key(uint32_t k) { w2 = (w2 & 0xffffu) | k << 16; }
};
constexpr uint32_t kInlineSlot = 0x40000000u;  // | which << 26 | parent

struct GstLds {
    u32x4 root[256];
    uint32_t doc_base[kDocCache + 1];
};

struct GstWave {
    // shard arena
    // The shard arena is reached through buffer resources: a wave-uniform byte offset
    // rides in the instruction's scalar offset (one s_lshl per access instead of
    // 64-bit address arithmetic) and the section offsets sit in VGPRs (vreg).
    //   nodes: 2 x uint4 per node: {link, cnt, e0.w0, e0.w1}, {e0.w2, e1.w0, e1.w1, e1.w2}
    __amdgpu_buffer_rsrc_t ar;  // shard arena: doc starts, nodes, child-map hash
    __amdgpu_buffer_rsrc_t tr;  // live chunk text
    uint32_t v_doc, v_nodes, v_hash, v_hash4, v_zero, v_lane, v_lane4;  // VGPRs
    // lookup candidates: the child count lane l's candidate needs (lane 0/1: inline
    // child 0/1, lanes 4..7: bucket entries, others never) and whether it is inline
    uint32_t v_need, v_inl;
    uint32_t kc_off, kc_key;  // canonise's cached first key (valid within one split loop)
    uint32_t node_cap, hash_mask, doc_cap;
    PX_LAS GstLds *lds;
    // persistent counters
    uint32_t n_nodes, n_docs, chunk_seq, epoch, status;
    int32_t pools, used, pool_open;
    uint64_t ctext_off;
    uint32_t ub;  // this launch's UB reads (added to the shard's 64-bit total at the end)
    // current doc + its byte window (lane l holds bytes [wb + 4l, wb + 4l + 4))
    uint32_t cur, cur_base, cur_len, wb, win;
    // active point (SuffixTree.h:33-40); act_base/act_len: text extent of act_doc
    // i: the doc byte being inserted (the reference's `counter`)
    uint32_t act_node, act_doc, act_direct, act_off, i, act_base, act_len;
    int32_t remainder;
    PX_GAS uint32_t *msg;  // the current doc's encoder messages
#ifdef PX_PROFILE
    uint64_t prof[P_N];
#endif

    PX_DEV uint32_t ldt(uint32_t vo, uint32_t rel) const {  // text byte at vo + rel
        return __builtin_amdgcn_raw_buffer_load_b8(tr, (int)(vo + rel), 0, 0);
    }
    PX_DEV uint32_t tbyte(uint32_t rel) const { return uni(ldt(v_zero, rel)); }
    // offsets are formed on the vector unit (v_lshl_add into the voffset operand): the
    // scalar unit, which the walk saturates, only supplies the node id
    PX_DEV u32x4 nld(uint32_t n, uint32_t h) const {  // half h of node n's record
        return __builtin_amdgcn_raw_buffer_load_b128(ar, (int)(v_nodes + n * 32u + h * 16u), 0, 0);
    }
    PX_DEV uint32_t nlink(uint32_t n) const {
        return __builtin_amdgcn_raw_buffer_load_b32(ar, (int)(v_nodes + n * 32u), 0, 0);
    }
    PX_DEV void nst(uint32_t n, uint32_t h, u32x4 v) {
        __builtin_amdgcn_raw_buffer_store_b128(v, ar, (int)(v_nodes + n * 32u + h * 16u), 0, 0);
    }
    PX_DEV void nstw(uint32_t n, uint32_t w, uint32_t v) {  // word w of node n's record
        __builtin_amdgcn_raw_buffer_store_b32(v, ar, (int)(v_nodes + n * 32u + w * 4u), 0, 0);
    }
    PX_DEV u32x4 hld(uint32_t b) const {  // bucket b: lane l holds entry 4b + (l & 3)
        return __builtin_amdgcn_raw_buffer_load_b128(ar, (int)(v_hash4 + b * 64u), 0, 0);
    }
    PX_DEV void hst(uint32_t slot, u32x4 v) {
        __builtin_amdgcn_raw_buffer_store_b128(v, ar, (int)(v_hash + slot * 16u), 0, 0);
    }
    PX_DEV uint32_t dld(uint32_t d) const {
        return __builtin_amdgcn_raw_buffer_load_b32(ar, (int)(v_doc + d * 4u), 0, 0);
    }
    PX_DEV void dst(uint32_t d, uint32_t v) { __builtin_amdgcn_raw_buffer_store_b32(v, ar, (int)(v_doc + d * 4u), 0, 0); }
    PX_DEV void set_text(PX_GAS uint8_t *p) {
        tr = __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, 0x7fffffff, 0x00020000);
    }

    PX_DEV void fail(uint32_t code) {
        if (status == kOk) status = code;
    }

    // MemPool::p_malloc block accounting (MemPool.cpp:7-37)
    // The pool is always open while docs are encoded (clear_tree's root node opens
    // it), so the hot path is the branch-free "next pool when the request does not fit".
    PX_DEV void charge(int32_t blocks) {
        const int32_t t = used + blocks;
        const bool next = t > kPoolBlocks;
        pools += (int32_t)next;
        used = next ? blocks : t;
    }
    PX_DEV void charge_first(int32_t blocks) {  // MemPool's first p_malloc opens pool 1
        pool_open = 1;
        pools = 1;
        used = blocks;
    }

    // ---- doc extents: LDS cache for the first kDocCache docs
    PX_DEV uint32_t docbase(uint32_t d) const {
        return d <= kDocCache ? uni(lds->doc_base[d]) : uni(dld(d));
    }
    PX_DEV void set_docbase(uint32_t d, uint32_t v) {
        dst(d, v);
        if (d <= kDocCache) lds->doc_base[d] = v;
    }
    PX_DEV void set_act_doc(uint32_t d) {
        act_doc = d;
        act_base = docbase(d);
        act_len = docbase(d + 1) - act_base;
    }

    // ---- current doc window
    PX_DEV void load_window(uint32_t at) {
        uint32_t abs0 = (cur_base + at) & ~3u;  // 4-byte aligned window start
        wb = abs0 - cur_base;                    // may wrap below 0 (unsigned): range tests cope
        win = __builtin_amdgcn_raw_buffer_load_b32(tr, (int)v_lane4, (int)abs0, 0);
    }
    PX_DEV uint32_t curchar(uint32_t p) {  // byte p of the current doc
        uint32_t d = p - wb;
        if (d < kWin) return (readlane(win, d >> 2) >> ((d & 3) * 8)) & 0xffu;
        return tbyte(cur_base + p);
    }

    // byte the reference reads through strs[act_doc]->data[pos]; past the end it
    // reads heap bytes (UB) -> modelled as a value matching nothing, counted.
    PX_DEV int32_t stale_byte(uint32_t pos) {
        if (pos >= act_len) {
            ++ub;
            return -1;
        }
        return (int32_t)tbyte(act_base + pos);
    }


    // ---- child map
    PX_DEV static void unpack(uint32_t w0, uint32_t w1, uint32_t w2, Edge &e) {
        e.w0 = w0;
        e.w1 = w1;
        e.w2 = w2;
    }
    PX_DEV static uint32_t pk0(const Edge &e) { return e.w0; }
    PX_DEV static uint32_t pk1(const Edge &e) { return e.w1; }
    PX_DEV static uint32_t pk2(const Edge &e) { return e.w2; }

    // child of n keyed by byte c.  found: fills e.  not found: slot = where a new
    // child goes (kNone: a hash slot must still be probed) and ncnt = n's count.
    PX_DEV bool lookup(uint32_t n, uint32_t c, Edge &e, uint32_t &slot, uint32_t &ncnt) {
        if (n == kRoot) {
            u32x4 v = lds->root[c];
            slot = kRootSlot | c;
            ncnt = 3;
            if (uni(v.y) == kNone) return false;
            unpack(uni(v.y), uni(v.z), uni(v.w), e);
            e.slot = slot;
            return true;
        }
        PX_CNT(P_LOOKUPS, 1);
        const uint32_t lane = lane_id();
        const uint32_t nb = (hash_mask >> 2);
        // the bucket index is hashed on the vector unit (n forced into a VGPR), so the
        // scalar unit, which the walk saturates, only sees the result's uses
        const uint32_t vb = hslot(vreg(n), c) & nb;
        // the node record and the first hash bucket, issued together
        u32x4 r0 = nld(n, 0), r1 = nld(n, 1);
        u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ar, (int)(v_hash4 + vb * 64u), 0, 0);
        ncnt = uni(r0.y);
        const uint32_t want = n | (epoch << 26);
        {
            // one candidate per lane: lane 0 / 1 = inline child 0 / 1, lanes 4..7 = the
            // bucket's entries 0..3; a single ballot finds the child keyed c
            // (branch-free: every term is a per-lane vector value)
            const bool in0 = lane == 0, in1 = lane == 1;
            const uint32_t w0 = in0 ? r0.z : in1 ? r1.y : v.y;
            const uint32_t w1 = in0 ? r0.w : in1 ? r1.z : v.z;
            const uint32_t w2 = in0 ? r1.x : in1 ? r1.w : v.w;
            const uint32_t ok = (uint32_t)(ncnt >= v_need) & ((uint32_t)(v.x == want) | v_inl) &
                                (uint32_t)(((w2 >> 16) & 0xffu) == c);
            const uint64_t mm = ballot(ok != 0);
            if (mm) {
                const uint32_t l = ffs64(mm);
                unpack(readlane(w0, l), readlane(w1, l), readlane(w2, l), e);
                e.slot = slot = l < 2 ? (kInlineSlot | (l << 26) | n) : uni(vb) * kBucket + (l - 4);
                return true;
            }
        }
        if (ncnt < 2) {
            slot = kInlineSlot | (ncnt << 26) | n;
            return false;
        }
        uint32_t b = uni(vb);
        {
            // the bucket's first free entry, if any (for ncnt == 2 there are no hash entries yet)
            const uint64_t me = ballot(lane - 4u < 4u && (v.x >> 26) != epoch);
            if (me || ncnt == 2) {
                slot = me ? b * kBucket + (ffs64(me) - 4) : kNone;
                return false;
            }
        }
        // the first bucket is full of other parents' entries: probe on
        b = (b + 1) & nb;
        v = hld(b);
        for (uint32_t guard = 0; guard < nb; ++guard) {
            PX_CNT(P_PROBES, 1);
            bool valid = (v.x >> 26) == epoch;
            bool match = lane < kBucket && v.x == want && ((v.w >> 16) & 0xffu) == c;
            bool empty = lane < kBucket && !valid;
            uint64_t mm = ballot(match), me = ballot(empty);
            if (mm) {
                uint32_t l = ffs64(mm);
                unpack(readlane(v.y, l), readlane(v.z, l), readlane(v.w, l), e);
                e.slot = slot = b * kBucket + l;
                return true;
            }
            if (me) {
                slot = b * kBucket + ffs64(me);
                return false;
            }
            b = (b + 1) & nb;
            v = hld(b);
        }
        fail(kErrCapacity);
        slot = kNone;
        return false;
    }
    PX_DEV bool lookup(uint32_t n, uint32_t c, Edge &e) {
        uint32_t slot, ncnt;
        return lookup(n, c, e, slot, ncnt);
    }
    // a free hash slot for a new child of n (n already has >= 2 children)
    PX_DEV uint32_t hash_free_slot(uint32_t n, uint32_t c) {
        const uint32_t lane = lane_id();
        const uint32_t nb = (hash_mask >> 2);
        uint32_t b = hslot(n, c) & nb;
        for (uint32_t guard = 0; guard <= nb; ++guard) {
            PX_CNT(P_PROBES, 1);
            u32x4 v = hld(b);
            uint64_t me = ballot(lane < kBucket && (v.x >> 26) != epoch);
            if (me) return b * kBucket + ffs64(me);
            b = (b + 1) & nb;
        }
        fail(kErrCapacity);
        return kNone;
    }
    PX_DEV void write_entry(uint32_t slot, uint32_t parent, const Edge &e) {
        if (slot & kRootSlot) {
            lds->root[slot & 0xffu] = mk4(0, pk0(e), pk1(e), pk2(e));
        } else if (slot & kInlineSlot) {
            uint32_t n = slot & kNodeMask;
            const uint32_t o = (slot >> 26) & 1u ? 5 : 2;  // e1 at words 5..7, e0 at words 2..4
            typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
            __builtin_amdgcn_raw_buffer_store_b96(u32x3{pk0(e), pk1(e), pk2(e)}, ar, (int)v_nodes,
                                                  (int)(n * 32u + o * 4u), 0);
        } else if (slot != kNone) {
            hst(slot, mk4(parent | (epoch << 26), pk0(e), pk1(e), pk2(e)));
        }
    }
    // add a child that is known to be absent (charges one map entry).  hint: the free
    // slot a failed lookup(parent, kid.key) just found (kNone: probe for one)
    PX_DEV void add_child(uint32_t parent, uint32_t pcnt, const Edge &kid, uint32_t hint) {
        charge(kEdgeBlocks);
        uint32_t slot = pcnt < 2 ? (kInlineSlot | (pcnt << 26) | parent)
                                 : (hint != kNone ? hint : hash_free_slot(parent, kid.key()));
        write_entry(slot, parent, kid);
        if (parent != kRoot && pcnt < 3) nstw(parent, 1, pcnt + 1);
    }

    // capacity: encode_doc checks once per doc that 2 * len more nodes fit (a doc adds
    // at most one leaf per suffix and one inner node per leaf)
    PX_DEV bool new_node(uint32_t &id) {
        charge(kNodeBlocks);
        id = n_nodes++;
        return true;
    }

    // ---- fresh chunk (SuffixTree::init_prop, SuffixTree.cpp:61-78)
    PX_DEV void clear_tree() {
        const uint32_t lane = lane_id();
        n_nodes = 0;
        pools = 0;
        used = 0;
        pool_open = 0;
        for (uint32_t c = lane; c < 256; c += 64) lds->root[c] = mk4(0, kNone, 0, 0);
        if (++epoch > (uint32_t)kMaxEpoch) {  // epochs exhausted: really clear
            for (uint32_t s = 0; s <= hash_mask; s += 64)
                if (s + lane <= hash_mask)
                    __builtin_amdgcn_raw_buffer_store_b128(mk4(0, 0, 0, 0), ar, (int)(v_hash + lane * 16u), (int)(s * 16u), 0);
            epoch = 1;
        }
        wave_sync();
        charge_first(kNodeBlocks);  // the root (SuffixTree::init_prop)
        nst(n_nodes++, 0, mk4(kRoot, 0, 0, 0));
    }

    // ---- encoder messages (the PXSMsg stream SuffixTree::setitem hands to
    // PiXiuStr_init_stream, PiXiuStr.h:55-59, SuffixTree.cpp:291-304): one u32 per doc
    // byte, idx << 16 | pos for COMPRESS, kPassMsg for NO_COMPRESS.  The stream
    // encoder itself runs lane-parallel afterwards (k_gst_emit), so the walk carries
    // none of its state.  All lanes store the same word (no exec-mask juggling).
    PX_DEV void feed(bool is_c, uint32_t idx, uint32_t pos, uint32_t b) {
        PX_TRACE_MSG(is_c ? (int32_t)idx : -3, is_c ? pos : 0, b);
        msg[i] = is_c ? (idx << 16 | pos) : kPassMsg;
    }
    // m (<= 64) consecutive COMPRESS messages (idx, pos0 + k) for doc bytes at + k
    PX_DEV void feed_bulk(uint32_t at, uint32_t idx, uint32_t pos0, uint32_t m, uint64_t m251) {
#ifdef PX_TRACE
        for (uint32_t t = 0; t < m; ++t) PX_TRACE_MSG(idx, pos0 + t, ((m251 >> t) & 1) ? 251 : -1);
#endif
        if (lane_id() < m) msg[at + lane_id()] = (idx << 16) | (pos0 + lane_id());
    }

    // ---- Ukkonen step pieces (SuffixTree.cpp:144-289)
    PX_DEV bool new_leaf(Edge &leaf, uint32_t c) {
        uint32_t id;
        if (!new_node(id)) return false;
        nst(id, 0, mk4(kRoot, 0, 0, 0));  // link, child count
        leaf.set(id, 0, cur, i, cur_len, c);
        return true;
    }

    // case_root: returns true (and the edge) when the byte exists under the root
    PX_DEV bool at_root(uint32_t c, bool send, Edge &e) {
        uint32_t slot, ncnt;
        if (!lookup(kRoot, c, e, slot, ncnt)) {
            Edge leaf;
            if (!new_leaf(leaf, c)) return false;
            charge(kEdgeBlocks);
            write_entry(slot, kRoot, leaf);
            --remainder;
            if (send) feed(false, 0, 0, c);
            return false;
        }
        set_act_doc(e.doc());
        act_direct = e.from();
        act_off = (act_off + 1) & 0xffffu;
        if (send) feed(true, e.doc(), e.from(), c);
        return true;
    }

    PX_DEV bool must_lookup(uint32_t n, uint32_t c, Edge &e) {
        if (!lookup(n, c, e)) {
            if (status == kOk) fail(kErrRefCrash);  // the reference dereferences NULL here
            return false;
        }
        return true;
    }

    // overflow_fix: canonise the active point along the current text
    PX_DEV bool canonise(Edge &e) {
#ifdef PX_PROFILE
        uint64_t tk = __builtin_amdgcn_s_memtime();
        if ((i - act_off) - wb >= kWin) PX_CNT(P_KEYMISS, 1);
        uint32_t key0 = curchar(i - act_off);
        uint64_t tl = __builtin_amdgcn_s_memtime();
        prof[P_T_KEY] += tl - tk;
        bool ok0 = must_lookup(act_node, key0, e);
        prof[P_T_LOOK] += __builtin_amdgcn_s_memtime() - tl;
        if (!ok0) return false;
#else
        // the first key is text[i - act_off]: act_off rarely changes between the
        // iterations of one split loop, so the byte is kept (kc_off = its act_off)
        if (act_off != kc_off) {
            kc_key = curchar(i - act_off);
            kc_off = act_off;
        }
        if (!must_lookup(act_node, kc_key, e)) return false;
#endif
        uint32_t supply;
        while (act_off > (supply = e.to() - e.from())) {
            act_node = e.id();
            act_off = (act_off - supply) & 0xffffu;
            if (!must_lookup(act_node, curchar(i - act_off), e)) return false;
            act_direct = e.from();
            PX_CNT(P_CANON_LVL, 1);
        }
        return true;
    }

    // split_grow: `split` and the byte of e at the split point were computed by
    // the caller (their loads were issued before this function's stores)
    PX_DEV bool grow(Edge &e, uint32_t &last_inner, uint32_t c, bool split, uint32_t key_e, uint32_t hint) {
        Edge leaf;
#ifdef PX_PROFILE
        uint64_t tq = __builtin_amdgcn_s_memtime();
#endif
        if (!new_leaf(leaf, c)) return false;
        --remainder;
#ifdef PX_PROFILE
        {
            uint64_t t2 = __builtin_amdgcn_s_memtime();
            prof[P_G_T_LEAF] += t2 - tq;
            tq = t2;
        }
#endif
        if (split) {
            Edge in;
            uint32_t in_id;
            if (!new_node(in_id)) return false;
            if (last_inner != kNone) nstw(last_inner, 0, in_id);
            last_inner = uni(in_id);
            const uint32_t in_to = (e.from() + act_off) & 0xffffu;
            in.set(in_id, key_e != c ? 2 : 1, e.doc(), e.from(), in_to, e.key());
            write_entry(e.slot, act_node, in);  // replaces e under its first byte: no charge
            e.set_from(in_to);
            e.set_key(key_e);
            // inner->set_sub(edge); inner->set_sub(leaf): an equal key replaces
            charge(kEdgeBlocks);
            if (key_e != c) {
                charge(kEdgeBlocks);
                nst(in_id, 0, mk4(kRoot, 2, pk0(e), pk1(e)));
                nst(in_id, 1, mk4(pk2(e), pk0(leaf), pk1(leaf), pk2(leaf)));
                e.slot = kInlineSlot | in_id;
            } else {
                nst(in_id, 0, mk4(kRoot, 1, pk0(leaf), pk1(leaf)));
                nstw(in_id, 4, pk2(leaf));
                e.slot = kNone;  // e fell out of the tree (replaced under the same byte)
            }
#ifdef PX_PROFILE
            prof[P_G_T_SPLIT] += __builtin_amdgcn_s_memtime() - tq;
#endif
        } else {
            PX_CNT(P_G_NOSPLIT, 1);
            if (last_inner != kNone) nstw(last_inner, 0, e.id());
            last_inner = uni(e.id());
            add_child(e.id(), e.cnt(), leaf, hint);
            if (e.cnt() < 3) {
                e.w0 += 1u << 26;
                write_entry(e.slot, act_node, e);
            }
#ifdef PX_PROFILE
            prof[P_G_T_ADD] += __builtin_amdgcn_s_memtime() - tq;
#endif
        }
        return true;
    }

    // compare the current text from doc position i against the active edge's label
    // (read through the stale active doc, SuffixTree.cpp:171,184) and apply the
    // matching prefix as COMPRESS messages in bulk.  Returns matched length.
    PX_DEV uint32_t fast_forward(const Edge &e, uint32_t i) {
        const uint32_t lane = lane_id();
        uint32_t limit = min(e.to() - e.from() - act_off, cur_len - i);
        uint32_t m = 0;
        while (m < limit) {
            uint32_t w = min(64u, limit - m);
            uint32_t t = e.from() + act_off + m + lane;  // position in the active doc
            bool live = lane < w;
            uint32_t a = live ? ldt(v_lane, cur_base + i + m) : 0;
            bool oob = live && t >= act_len;
            uint32_t b = (live && !oob) ? ldt(v_lane, act_base + e.from() + act_off + m) : 0x100u;
            uint64_t mism = ballot(live && (oob || a != b));
            uint64_t m251 = ballot(live && a == kEsc);
            uint32_t got = mism ? ffs64(mism) : w;
            if (got) feed_bulk(i + m, e.doc(), e.from() + act_off + m, got, m251);
            m += got;
            if (mism) {
                if (readlane((uint32_t)oob, got)) ++ub;
                break;
            }
        }
        return m;
    }

    // SuffixTree::setitem for one doc of `len` bytes already in the arena
    PX_DEV void encode_doc(uint32_t len) {
        cur_len = len;
        remainder = 0;
        i = 0;
        act_node = kRoot;
        act_doc = act_direct = act_off = 0;
        act_base = docbase(0);
        act_len = docbase(1) - act_base;
        load_window(0);
        bool have_e = false;
        Edge e;
        if (n_nodes + 2 * len + 1 > min(node_cap, kMaxNodes)) fail(kErrCapacity);
        while (i < len && status == kOk) {
            if (i - wb >= kWin - 64 && i - wb < 0x80000000u) load_window(i >= 64 ? i - 64 : 0);
            const uint32_t c = curchar(i);
            PX_TRACE_STATE(0);
            PX_CNT(P_BYTES, 1);
            if (act_node == kRoot && act_off == 0) {
                PX_T0();
                ++remainder;
                have_e = at_root(c, true, e);
                ++i;
                PX_CNT(P_ROOT, 1);
                PX_T1(P_T_ROOT);
                continue;
            }
            if (!have_e) {
                PX_T0();
                int32_t key = stale_byte(act_direct);
                if (key < 0) {
                    fail(kErrRefCrash);  // get_sub(garbage) -> NULL deref in the reference
                    break;
                }
                if (!must_lookup(act_node, (uint32_t)key, e)) break;
                have_e = true;
                PX_T1(P_T_DERIVE);
            }
            // free slot for c under e.id found by a failed lookup (valid until the next hash write)
            uint32_t hint = kNone;
            if (e.from() + act_off == e.to()) {
                Edge n;
                PX_T0();
                uint32_t ncnt;
                bool wd = e.cnt() && lookup(e.id(), c, n, hint, ncnt);
                PX_T1(P_T_WALK);
                if (wd) {
                    PX_CNT(P_WALK, 1);
                    ++remainder;
                    act_node = e.id();
                    set_act_doc(n.doc());
                    act_direct = n.from();
                    act_off = 1;
                    feed(true, n.doc(), n.from(), c);
                    e = n;  // child(act_node, text[act_doc][act_direct]) == n
                    ++i;
                    continue;
                }
            } else if (e.from() + act_off < e.to()) {
                PX_T0();
                uint32_t m = fast_forward(e, i);
                PX_T1(P_T_FF);
                PX_CNT(P_FF_CALLS, 1);
                PX_CNT(P_FF_BYTES, m);
#ifdef PX_TRACE
                for (uint32_t k = 1; k < m; ++k) PX_TRACE_STATE(k);
#endif
                if (m) {
                    remainder += (int32_t)m;
                    act_off = (act_off + m) & 0xffffu;
                    i += m;
                    continue;
                }
            }
            // mismatch: emit PASS, then split/grow along suffix links
            PX_CNT(P_PASS, 1);
            PX_T0();
            ++remainder;
            feed(false, 0, 0, c);
            uint32_t last_inner = kNone;
            // e's own byte at the split point, when an earlier read already has it
            int32_t e_next = -1;
            // the suffix link of act_node is loaded one iteration ahead (next to the
            // previous end check), so an iteration costs two dependent round trips
            uint32_t lraw = act_node != kRoot ? nlink(act_node) : 0u;
            kc_off = kNone;
            while (remainder > 0) {
                PX_CNT(P_ITERS, 1);
#ifdef PX_PROFILE
                uint64_t tg = __builtin_amdgcn_s_memtime();
#endif
                const bool split = (!e.cnt() || e.to() - e.from() > 1) && e.from() + act_off != e.to();
                uint32_t key_e = 0;
                if (split) key_e = e_next >= 0 ? (uint32_t)e_next : tbyte(docbase(e.doc()) + e.from() + act_off);
                PX_CNT(P_K_CACHED, split && e_next >= 0 ? 1 : 0);
                PX_CNT(P_K_LOAD1, split && e_next < 0 && act_off == 1 ? 1 : 0);
                PX_CNT(P_K_LOADN, split && e_next < 0 && act_off != 1 ? 1 : 0);
                if (!grow(e, last_inner, c, split, key_e, split ? kNone : hint)) break;
                hint = kNone;
#ifdef PX_PROFILE
                prof[P_T_GROW] += __builtin_amdgcn_s_memtime() - tg;
                tg = __builtin_amdgcn_s_memtime();
#endif
                e_next = -1;
                if (act_node == kRoot) {  // STNode::is_inner(act_node) == (act_node != root) here
                    act_off = (act_off - 1) & 0xffffu;
                    act_direct = (act_direct + 1) & 0xffffu;
                    if (act_off > 0) {
                        if (!canonise(e)) break;
                    } else {
                        at_root(c, false, e);
                        break;
                    }
                } else {
                    PX_CNT(P_LINK, 1);
                    act_node = uni(lraw);
                    if (!canonise(e)) break;
                }
#ifdef PX_PROFILE
                prof[P_T_CANON] += __builtin_amdgcn_s_memtime() - tg;
#endif
#ifdef PX_PROFILE
                tg = __builtin_amdgcn_s_memtime();
#endif
                // next iteration's suffix link, issued before this end check's wait
                lraw = act_node != kRoot ? nlink(act_node) : 0u;
                PX_CNT(P_E_LOOK, e.from() + act_off == e.to() ? 1 : 0);
                PX_CNT(P_E_OFF1, e.from() + act_off < e.to() && act_off == 1 ? 1 : 0);
                PX_CNT(P_E_OFF2, e.from() + act_off < e.to() && act_off == 2 ? 1 : 0);
                PX_CNT(P_E_OFF3, e.from() + act_off < e.to() && act_off == 3 ? 1 : 0);
                PX_CNT(P_E_OFF4P, e.from() + act_off < e.to() && act_off >= 4 ? 1 : 0);
                if (e.from() + act_off == e.to()) {
                    Edge n;
                    uint32_t ncnt;
                    if (e.cnt() && lookup(e.id(), c, n, hint, ncnt)) {
                        act_node = e.id();
                        set_act_doc(n.doc());
                        act_direct = n.from();
                        act_off = 1;
                        if (last_inner != kNone) nstw(last_inner, 0, act_node);
                        break;
                    }
                } else if (e.from() + act_off < e.to()) {
                    uint32_t ch = tbyte(docbase(e.doc()) + e.from() + act_off);
                    if (c == ch) {
                        act_off = (act_off + 1) & 0xffffu;
                        break;
                    }
                    e_next = (int32_t)ch;
                }
#ifdef PX_PROFILE
                prof[P_T_END] += __builtin_amdgcn_s_memtime() - tg;
#endif
            }
            PX_T1(P_T_SPLIT);
            have_e = false;
            ++i;
        }
    }
};

// kGstWaves independent shard waves per block: a CU holds at most 16 blocks, so
// one-wave blocks would cap residency at 4,096 waves chip-wide
constexpr uint32_t kGstWaves = 4;

__global__ void __launch_bounds__(64 * kGstWaves, 6) k_gst_encode(const GstShard *shards, uint32_t n_shards,
                                                   const uint32_t *doc_len, uint8_t *const *comp_dst,
                                                   const uint8_t *comp_base, uint32_t *msgs, uint32_t *rec_chunk,
                                                   uint32_t *rec_idx, uint32_t *rec_status, ShardState *st_out,
                                                   uint32_t *sink) {
    __shared__ GstLds lds_w[kGstWaves];
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint32_t s = blockIdx.x * kGstWaves + wv;
    if (s >= n_shards) return;
    GstLds &lds = lds_w[wv];
    const uint32_t lane = lane_id();
    const GstShard sh = shards[s];
    ShardState st = *sh.st;
    GstWave g;
    {
        const uint8_t *arena = (const uint8_t *)sh.st;  // the arena starts with the shard state
        g.ar = __builtin_amdgcn_make_buffer_rsrc((void *)arena, 0, 0x7fffffff, 0x00020000);
        g.v_doc = vreg((uint32_t)((const uint8_t *)sh.doc_base - arena));
        g.v_nodes = vreg((uint32_t)((const uint8_t *)sh.nodes - arena));
        g.v_hash = vreg((uint32_t)((const uint8_t *)sh.hash - arena));
        g.v_hash4 = g.v_hash + (lane & 3u) * 16u;
        g.v_zero = vreg(0);
        g.v_lane = lane;
        g.v_lane4 = lane * 4u;
        g.v_need = lane == 0 ? 1u : lane == 1 ? 2u : lane - 4u < 4u ? 3u : 4u;
        g.v_inl = lane < 2 ? 1u : 0u;
    }
    g.node_cap = sh.node_cap;
    g.hash_mask = sh.hash_mask;
    g.doc_cap = sh.doc_cap;
    g.lds = (PX_LAS GstLds *)&lds;
    g.n_nodes = uni(st.n_nodes);
    g.n_docs = uni(st.n_docs);
    g.chunk_seq = uni(st.chunk_seq);
    g.epoch = uni(st.epoch);
    g.status = uni(st.status);
    g.pools = unii(st.pools);
    g.used = unii(st.used_blocks);
    g.pool_open = unii(st.pool_open);
    g.ctext_off = uni64(st.ctext_off);
    g.ub = 0;
    g.set_text((PX_GAS uint8_t *)sh.text + g.ctext_off);
#ifdef PX_PROFILE
    for (int k = 0; k < P_N; ++k) g.prof[k] = 0;
    uint64_t t_kernel0 = __builtin_amdgcn_s_memtime();
#endif
    // stage the persistent root entries and doc starts into LDS
    for (uint32_t c = lane; c < 256; c += 64) lds.root[c] = ((const PX_GAS u32x4 *)sh.root)[c];
    for (uint32_t d = lane; d <= kDocCache; d += 64)
        lds.doc_base[d] = d <= max(g.n_docs, sh.replay) ? sh.doc_base[d] : 0;
    wave_sync();
    if (g.epoch == 0) {  // brand-new shard
        g.clear_tree();
        g.set_docbase(0, 0);
        g.n_docs = 0;
    }
    // a live chunk whose docs were encoded by the suffix-array path (px_psa.hip) has no
    // tree: re-walk its docs first (their messages go to a sink), then continue
    for (uint32_t d = 0; d < sh.replay && g.status == kOk; ++d) {
        g.cur = d;
        g.cur_base = g.docbase(d);
        const uint32_t len = g.docbase(d + 1) - g.cur_base;
        g.msg = (PX_GAS uint32_t *)sink;
        g.encode_doc(len);
        ++g.n_docs;
    }
    for (uint32_t r = sh.r0; r < sh.r1; ++r) {
        const uint32_t len = uni(doc_len[r]);
        if (g.status != kOk || len == 0xffffffffu) {
            if (lane == 0) {
                rec_status[r] = g.status != kOk ? g.status : (uint32_t)kErrInval;
            }
            continue;
        }
        // rotation (PiXiuCtrl.cpp:13-25): before the doc, by pool count or slot count
        if (g.pools >= kRotatePools || g.n_docs == (uint32_t)kChunkSlots) {
            uint32_t shift = g.docbase(g.n_docs);
            g.ctext_off += shift;
            g.set_text((PX_GAS uint8_t *)sh.text + g.ctext_off);
            g.n_docs = 0;
            g.set_docbase(0, 0);
            ++g.chunk_seq;
            g.clear_tree();
        }
        if (g.n_docs >= g.doc_cap) {
            g.fail(kErrCapacity);
            if (lane == 0) rec_status[r] = g.status;
            continue;
        }
        g.cur = g.n_docs;
        g.cur_base = g.docbase(g.cur);
        g.set_docbase(g.cur + 1, g.cur_base + len);
        wave_sync();
        g.msg = (PX_GAS uint32_t *)msgs + (comp_dst[r] - comp_base);
        g.encode_doc(len);
        ++g.n_docs;
        if (lane == 0) {
            rec_chunk[r] = g.chunk_seq;
            rec_idx[r] = g.cur;
            rec_status[r] = g.status;
        }
    }
    wave_sync();
#ifdef PX_PROFILE
    g.prof[P_T_TOTAL] = __builtin_amdgcn_s_memtime() - t_kernel0;
    if (lane == 0)
        for (int k = 0; k < P_N; ++k) atomicAdd(&g_prof[k], (unsigned long long)g.prof[k]);
#endif
    for (uint32_t c = lane; c < 256; c += 64) ((PX_GAS u32x4 *)sh.root)[c] = lds.root[c];
    if (lane == 0) {
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
        o.ub_reads = sh.st->ub_reads + g.ub;
        *sh.st = o;
        st_out[s] = o;  // compact copy: the host reads every shard's state in one transfer
    }
}

// ====================================================================== stream encoder
// PiXiuStr_init_stream (PiXiuStr.cpp:16-118) over one doc's message stream, one wave
// per record, 64 messages per step.  The sequential encoder is restated as
// per-position rules that lanes evaluate independently:
//   * 251 look-ahead (:33-54): a doc byte 251 that is not itself the second byte of
//     a pair starts a pair with its successor (in an escaped doc these are the escape
//     pairs); both messages of a pair are COMPRESS only if both were, else both PASS.
//   * a run = maximal sequence of (effective) COMPRESS messages; it ends at its last
//     message, whose idx and pos + 1 are the token's idx and `to` (:84-88, :112-115).
//   * try_explode (:56-82): a run of len > 6 becomes [251, len, idx:2, to:2] (len <= 255;
//     len 251 aliases the escape, kept) or [251, 1, idx:2, to:2, from:2]; shorter runs
//     and PASS messages are their doc bytes, literally.
// Output offsets come from a wave prefix sum of the per-position output sizes; the
// open run, the pair parity and the output cursor carry between steps.
// toks (optional): every record token it writes, in order, at toks + tok_off[r] (room for
// doc_len / 7 + 2), their count in ntok[r] (| kTokBad where the bytes must be parsed instead: a
// run of length 251, whose length byte reads as an escape pair -- the reference's alias --, a
// `from` that wraps below 0, a corrupt or failed record).
__global__ void __launch_bounds__(256) k_gst_emit(uint32_t n, const uint8_t *const *doc_ptr, const uint32_t *doc_len,
                                                  uint8_t *const *comp_dst, const uint8_t *comp_base,
                                                  const uint32_t *msgs, uint32_t *rec_status, uint32_t *comp_len,
                                                  const uint64_t *tok_off, TokEnt *toks, uint32_t *ntok) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    const uint64_t below = (1ull << lane) - 1;
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        const uint32_t len = uni(doc_len[r]);
        if (len == 0xffffffffu || uni(rec_status[r]) != kOk) {
            if (lane == 0) {
                comp_len[r] = 0;
                if (ntok) ntok[r] = kTokBad;
            }
            continue;
        }
        PX_GAS TokEnt *tk = toks ? (PX_GAS TokEnt *)toks + uni64(tok_off[r]) : nullptr;
        uint32_t ntk = 0;
        bool tbad = false;
        const PX_GAS uint8_t *doc = (const PX_GAS uint8_t *)doc_ptr[r];
        PX_GAS uint8_t *out = (PX_GAS uint8_t *)comp_dst[r];
        const PX_GAS uint32_t *msg = (const PX_GAS uint32_t *)msgs + (comp_dst[r] - comp_base);
        uint32_t outp = 0;
        bool second_in = false;  // position ws is the second byte of a pair
        bool prevc_in = false;   // raw COMPRESS-ness of position ws - 1
        uint32_t open_start = 0; // first position of the run open at ws (== ws: none)
        uint32_t open_msg = 0;   // message at ws - 1 (the open run's last so far)
        bool corrupt = false;
        // a run's output at o: a token, or its doc bytes when it is 6 or shorter
        auto run_out = [&](uint32_t o, uint32_t rl, uint32_t m, uint32_t start) {
            if (rl > 6) {
                const uint32_t idx = m >> 16, to = ((m & 0xffffu) + 1u) & 0xffffu;
                out[o] = kEsc;
                out[o + 1] = rl > 255 ? kBigSign : (uint8_t)rl;
                out[o + 2] = (uint8_t)idx;
                out[o + 3] = (uint8_t)(idx >> 8);
                out[o + 4] = (uint8_t)to;
                out[o + 5] = (uint8_t)(to >> 8);
                if (rl > 255) {
                    const uint32_t from = (to - rl) & 0xffffu;
                    out[o + 6] = (uint8_t)from;
                    out[o + 7] = (uint8_t)(from >> 8);
                }
            } else {
                for (uint32_t j = 0; j < rl; ++j) out[o + j] = doc[start + j];
            }
        };
        auto run_size = [](uint32_t rl) -> uint32_t { return rl > 6 ? (rl > 255 ? 8u : 6u) : rl; };
        // each window's doc bytes and messages are loaded two windows ahead (a step needs the
        // next window's first message, and a step is shorter than a load's latency)
        uint32_t bn = lane < len ? doc[lane] : 0u, mn = lane < len ? msg[lane] : kPassMsg;
        uint32_t bn2 = 64 + lane < len ? doc[64 + lane] : 0u, mn2 = 64 + lane < len ? msg[64 + lane] : kPassMsg;
        for (uint32_t ws = 0; ws < len; ws += 64) {
            const uint32_t k = ws + lane;
            const bool live = k < len;
            const uint32_t b = bn, m = mn;
            bn = bn2;
            mn = mn2;
            bn2 = ws + 128 + lane < len ? doc[ws + 128 + lane] : 0u;
            mn2 = ws + 128 + lane < len ? msg[ws + 128 + lane] : kPassMsg;
            const bool isc = m != kPassMsg;
            const uint64_t cm = ballot(isc);
            const bool nextc_63 = ws + 64 < len && uni(readlane(mn, 0)) != kPassMsg;
            const bool isc_next = lane < 63 ? ((cm >> (lane + 1)) & 1) != 0 : nextc_63;
            const bool isc_prev = lane > 0 ? ((cm >> (lane - 1)) & 1) != 0 : prevc_in;
            // pair starts: within a run of 251 bytes they alternate from the run's start
            const uint64_t non251 = ~ballot(live && b == kEsc);
            const uint64_t nb = non251 & below;
            const uint32_t rlen = nb ? lane - (64u - (uint32_t)__clzll((long long)nb)) : lane + (second_in ? 1u : 0u);
            const bool ps = live && b == kEsc && (rlen & 1u) == 0;
            const uint64_t psm = ballot(ps);
            const bool sec = lane > 0 ? ((psm >> (lane - 1)) & 1) != 0 : second_in;
            if (ballot(ps && k + 1 >= len)) corrupt = true;  // stream ends inside a pair
            const bool effc = isc && (ps ? isc_next : sec ? isc_prev : true);
            const uint64_t em = ballot(live && effc);
            // a run ending at lane 63 is only known to end with the doc; otherwise it
            // stays open and the next step's lane 0 emits it if that lane breaks it
            const bool end = effc && (lane < 63 ? ((em >> (lane + 1)) & 1) == 0 : k + 1 >= len);
            const bool flush_prev = lane == 0 && open_start < ws && !effc;
            const uint64_t nc = ~em & below;
            const uint32_t start = nc ? ws + (64u - (uint32_t)__clzll((long long)nc)) : open_start;
            const uint32_t rl = k + 1 - start;
            const uint32_t pre = flush_prev ? run_size(ws - open_start) : 0u;
            uint32_t size = pre;
            if (live && !effc) size += 1;
            if (end) size += run_size(rl);
            const int32_t incl = wave_incl_scan_dpp((int32_t)size);
            uint32_t o = outp + (uint32_t)incl - size;
            if (tk) {  // the step's record tokens, in output order (lane 0's flushed run comes first)
                uint32_t tx = 0, tl = 0, tm = 0, tof = 0;
                bool has = false;
                if (flush_prev && ws - open_start > 6) {
                    has = true;
                    tx = open_start;
                    tl = ws - open_start;
                    tm = open_msg;
                    tof = o;
                } else if (end && rl > 6) {
                    has = true;
                    tx = start;
                    tl = rl;
                    tm = m;
                    tof = o + pre;
                }
                const uint64_t hm = ballot(has);
                if (has) {
                    const uint32_t to = ((tm & 0xffffu) + 1u) & 0xffffu, from = (to - tl) & 0xffffu;
                    tbad = tbad || tl == 251u || to < tl;
                    *(PX_GAS u32x4 *)(tk + ntk + (uint32_t)__popcll(hm & below)) =
                        mk4(tx, tof, (tm >> 16) | from << 16, tl | (tl > 255 ? 8u : 6u) << 16);
                }
                ntk += (uint32_t)__popcll(hm);
            }
            if (flush_prev) {
                run_out(o, ws - open_start, open_msg, open_start);
                o += pre;
            }
            if (live && !effc) out[o] = (uint8_t)b;
            if (end) run_out(o, rl, m, start);
            outp += uni(readlane((uint32_t)incl, 63));
            second_in = (psm >> 63) & 1;
            prevc_in = (cm >> 63) & 1;
            open_start = ((em >> 63) & 1) ? uni(readlane(start, 63)) : ws + 64;
            open_msg = uni(readlane(m, 63));
        }
        tbad = ballot(tbad) != 0;
        if (lane == 0) {
            comp_len[r] = outp;
            if (corrupt) rec_status[r] = kErrCorrupt;
            if (ntok) ntok[r] = ntk | (tbad || corrupt ? kTokBad : 0u);
        }
    }
}

// ====================================================================== setup
// Zero the child map and the state of every brand-new shard arena (one launch per
// batch instead of a memset and a copy per shard).
__global__ void __launch_bounds__(256) k_shard_init(uint32_t n, const ShardInit *jobs) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t j = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); j < n; j += waves) {
        const ShardInit job = jobs[j];
        PX_GAS u32x4 *h = (PX_GAS u32x4 *)job.hash;
        for (uint64_t k = lane; k < job.entries; k += 64) h[k] = mk4(0, 0, 0, 0);
        PX_GAS u32x4 *st = (PX_GAS u32x4 *)job.st;
        if (lane < sizeof(ShardState) / 16) st[lane] = mk4(0, 0, 0, 0);
    }
}

// Write new chunk-table entries (one transfer + one launch per batch).
__global__ void __launch_bounds__(256) k_scatter_slots(uint32_t n, const SlotPut *puts) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const PX_GAS u32x4 *src = (const PX_GAS u32x4 *)&puts[i].val;
    PX_GAS u32x4 *dst = (PX_GAS u32x4 *)puts[i].dst;
    dst[0] = src[0];
    dst[1] = src[1];
    dst[2] = src[2];
}

// The batch's slots into their chunks' device tables, with the segment counts k_tokenize
// found (px_runtime.cpp set_nseg's rule), and each record's link job (a no-op job for a
// record that was not placed).  Replaces a host-built table of (destination, slot) pairs.
__global__ void __launch_bounds__(256) k_slot_place(uint32_t n, const RecSlot *src, const uint32_t *tok,
                                                    const SlotDst *d, LinkJob *jobs) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const SlotDst sd = d[r];
    if (!sd.dst) {
        jobs[r] = LinkJob{nullptr, nullptr, nullptr, 0u, 0u};
        return;
    }
    RecSlot s = src[r];
    const uint32_t t = tok[r];
    s.nseg = t & ~(1u << 31);  // (bit 31: k_tokenize's kNoPidx, no position index)
    if (t >> 31) {
        s.pidx_n = 0;
        s.lane = nullptr;
    }
    *sd.dst = s;
    jobs[r] = LinkJob{const_cast<SegEnt *>(s.seg), const_cast<LaneEnt *>(s.lane), sd.dst - sd.idx, s.nseg, sd.nrec};
}

// ====================================================================== store
// Copy each record's compressed bytes from scratch into the packed store.
__global__ void __launch_bounds__(256) k_compact(uint32_t n, uint8_t *const *src, const uint32_t *len,
                                                 uint8_t *dst, const uint64_t *dst_off) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        const PX_GAS uint8_t *s = (const PX_GAS uint8_t *)src[r];
        PX_GAS uint8_t *d = (PX_GAS uint8_t *)dst + dst_off[r];
        uint32_t l = len[r];
        for (uint32_t o = lane; o < l; o += 64) d[o] = s[o];
    }
}

// 251 bytes per compressed record: bounds its segment count (2 * n + 1, + sentinel)
__global__ void __launch_bounds__(256) k_count_esc(uint32_t n, uint8_t *const *src, const uint32_t *len,
                                                   uint32_t *n_esc) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        const PX_GAS uint8_t *s = (const PX_GAS uint8_t *)src[r];
        const uint32_t l = len[r];
        uint32_t cnt = 0;
        for (uint32_t o = lane; o < l; o += 64) cnt += s[o] == kEsc;
        for (int k = 32; k > 0; k >>= 1) cnt += __shfl_xor(cnt, k);
        if (lane == 0) n_esc[r] = cnt;
    }
}

// Segment index over the token grammar of PXSGen (PiXiuStr.h:139-192): one SegEnt
// (px_common.h) per segment, then an end sentinel {src_total, src_total, comp_len | 3 << 30}.
// Kinds: 0 plain (literals and 251-pairs, copied verbatim), 1 skip (251 + 3..6: no
// source bytes), 2 record, 3 end.  pidx[b] = the segment holding source position 16b.
// A record whose source positions are not monotone (a record token with to < from)
// gets no position index (nseg_out bit 31) and is only decoded by the serial path.
constexpr uint32_t kSegRecord = 2u << 30, kSegSkip = 1u << 30, kSegEnd = 3u << 30, kSegMask = (1u << 30) - 1;
constexpr uint32_t kNoPidx = 1u << 31;

PX_DEV void put_ent(PX_GAS SegEnt *seg, uint32_t k, u32x4 lo) { *(PX_GAS u32x4 *)(seg + k) = lo; }

__global__ void __launch_bounds__(256) k_tokenize(uint32_t n, const RecSlot *slots_in, uint32_t *nseg_out,
                                                  uint32_t *status, const uint32_t *ntok) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        if (ntok && !(uni(ntok[r]) & kTokBad)) continue;  // (k_tok_segs built it from the encoder's tokens)
        const RecSlot sl = slots_in[r];
        if (!sl.seg) {  // (room for lane entries only: k_tok_segs had to take it -- cannot happen)
            if (lane_id() == 0) {
                nseg_out[r] = 0;
                status[r] = kErrCorrupt;
            }
            continue;
        }
        const PX_GAS uint8_t *comp = (const PX_GAS uint8_t *)sl.comp;
        const uint64_t comp_addr = (uint64_t)sl.comp;
        const uint32_t len = sl.comp_len;
        PX_GAS SegEnt *seg = (PX_GAS SegEnt *)sl.seg;
        PX_GAS uint16_t *pidx = (PX_GAS uint16_t *)sl.pidx;
        PX_GAS LaneEnt *lanes = (PX_GAS LaneEnt *)sl.lane;
        const uint32_t pidx_n = sl.pidx_n, cap = sl.seg_cap ? sl.seg_cap : 0xffffffffu;
        uint32_t ns = 0, p = 0, wb = 0, err = 0, plain_start = 0;
        int32_t src = 0, plain_src = 0;
        bool plain_open = false, mono = true, have = false, over = false;
        uint32_t pend_x = 0, pend_z = 0, pend_w = 0;
        // the pending segment is written once the next one starts (its end is then known)
        auto emit = [&](int32_t x, uint32_t z, uint32_t w) {
            if (have) {
                if (ns + 1u >= cap) {  // (no room for it and the sentinel: the record fails)
                    over = true;
                    ++ns;
                    pend_x = (uint32_t)x;
                    pend_z = z;
                    pend_w = w;
                    return;
                }
                if (lane == 0) {
                    put_ent(seg, ns, mk4(pend_x, (uint32_t)x, pend_z, pend_w));
                    if (lanes) {
                        const int64_t d = (int64_t)comp_addr - (int64_t)(uint64_t)(lanes + ns);
                        const int32_t rel = (pend_z >> 30) == 0 ? (int32_t)(d >> 3) : kRelNone;
                        *(PX_GAS u32x4 *)(lanes + ns) = mk4(pend_x | (uint32_t)x << 16, pend_z, pend_w, (uint32_t)rel);
                    }
                }
                // lane entries need 16-bit coordinates and a comp base within +-16 GiB
                const int64_t dz = (int64_t)comp_addr - (int64_t)(uint64_t)(lanes + ns);
                if (lanes && (dz >> 3) != (int64_t)(int32_t)(dz >> 3)) mono = false;
                if (x < (int32_t)pend_x || x > 0xffff) {
                    mono = false;
                } else if (mono && pidx_n) {
                    uint32_t b0 = (pend_x + 15) >> 4, b1 = min(((uint32_t)x + 15) >> 4, pidx_n);
                    for (uint32_t b = b0 + lane; b < b1; b += 64) pidx[b] = (uint16_t)ns;
                }
                ++ns;
            }
            pend_x = (uint32_t)x;
            pend_z = z;
            pend_w = w;
            have = true;
        };
        // aligned 64-byte windows, [wb, wb + 64) in b and the next ones in bn, b2, b3: a token
        // starting in the first is wholly inside the first two, and each window's load is
        // issued three windows ahead (a window is consumed faster than one load's latency)
        uint32_t b = lane < len ? comp[lane] : 0;
        uint32_t bn = 64 + lane < len ? comp[64 + lane] : 0;
        uint32_t b2 = 128 + lane < len ? comp[128 + lane] : 0;
        uint32_t b3 = 192 + lane < len ? comp[192 + lane] : 0;
        auto byte_at = [&](uint32_t q) -> uint32_t {  // q < wb + 128
            const uint32_t d = q - wb;
            const uint32_t r0 = readlane(b, d & 63u), r1 = readlane(bn, d & 63u);
            return d < 64 ? r0 : r1;
        };
        while (p < len) {
            while (p >= wb + 64) {
                wb += 64;
                b = bn;
                bn = b2;
                b2 = b3;
                b3 = wb + 192 + lane < len ? comp[wb + 192 + lane] : 0;
            }
            if (!plain_open) {
                plain_open = true;
                plain_start = p;
                plain_src = src;
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
            if (p + 1 >= len) {
                err = kErrCorrupt;
                break;
            }
            uint32_t nx = byte_at(p + 1);
            if (nx == kKeyEnd || nx == kEsc || nx == kValEnd) {
                p += 2;
                src += 2;
                continue;
            }
            // record or skip token: closes the plain segment (dropped if empty)
            if (plain_start < p) emit(plain_src, plain_start, 0);
            if (nx == kBigSign || nx > 6) {
                uint32_t size = nx == kBigSign ? 8u : 6u;
                if (p + size > len) {
                    err = kErrCorrupt;
                    break;
                }
                uint32_t idx = byte_at(p + 2) | (byte_at(p + 3) << 8);
                uint32_t to = byte_at(p + 4) | (byte_at(p + 5) << 8);
                uint32_t from = nx == kBigSign ? (byte_at(p + 6) | (byte_at(p + 7) << 8)) : ((to - nx) & 0xffffu);
                emit(src, p | kSegRecord, idx | from << 16);
                src += (int32_t)to - (int32_t)from;
                p += size;
            } else {
                emit(src, p | kSegSkip, 0);
                p += 1;
            }
            plain_open = false;
        }
        if (!err) {
            if (plain_open && plain_start < len) emit(plain_src, plain_start, 0);
            emit(src, len | kSegEnd, 0);  // closes the last segment; the sentinel stays pending
            if (over) err = kErrCorrupt;
        }
        if (!err) {
            if (lane == 0) {
                put_ent(seg, ns, mk4((uint32_t)src, (uint32_t)src, len | kSegEnd, 0));
                if (lanes) *(PX_GAS u32x4 *)(lanes + ns) = mk4((uint32_t)src | (uint32_t)src << 16, len | kSegEnd, 0, 0);
            }
            // blocks past the source end: no segment
            if (mono && pidx_n)
                for (uint32_t k = ((uint32_t)max(src, 0) + 15) / 16 + lane; k < pidx_n; k += 64)
                    pidx[k] = (uint16_t)min(ns, 65535u);
        }
        if (lane == 0) {
            nseg_out[r] = err ? 0 : (ns | (mono && pidx_n ? 0u : kNoPidx));
            status[r] = err;
        }
    }
}

// The segment index of a record from the tokens k_gst_emit wrote (the same entries k_tokenize
// parses out of the compressed bytes: plain segments between the record tokens, each token
// covering its run's doc positions, then the end sentinel), 64 tokens per step, one wave per
// record.  Records flagged kTokBad are left to k_tokenize (launched after it), and so is a
// record whose stored bytes do not hold its tokens (a record not placed: comp_len 0).
__global__ void __launch_bounds__(256) k_tok_segs(uint32_t n, const RecSlot *slots_in, const uint32_t *doc_len,
                                                  const uint64_t *tok_off, const TokEnt *toks, uint32_t *ntok,
                                                  uint32_t *nseg_out, uint32_t *status) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < n; r += waves) {
        const uint32_t nt = uni(ntok[r]);
        if (nt & kTokBad) continue;
        const RecSlot sl = slots_in[r];
        const uint64_t comp_addr = uni64((uint64_t)sl.comp);
        const uint32_t clen = uni(sl.comp_len), L = uni(doc_len[r]), pidx_n = uni(sl.pidx_n);
        PX_GAS SegEnt *seg = (PX_GAS SegEnt *)uni64((uint64_t)sl.seg);
        PX_GAS uint16_t *pidx = (PX_GAS uint16_t *)uni64((uint64_t)sl.pidx);
        PX_GAS LaneEnt *lanes = (PX_GAS LaneEnt *)uni64((uint64_t)sl.lane);
        const PX_GAS TokEnt *tk = (const PX_GAS TokEnt *)toks + uni64(tok_off[r]);
        bool fits = clen > 0 && L <= 0xffffu && (!sl.seg_cap || 2u * nt + 2u <= sl.seg_cap);
        if (fits && nt) {
            const u32x4 t = *(const PX_GAS u32x4 *)(tk + nt - 1);  // (tokens come in comp order: x, o, w, rs)
            fits = t.y + (t.w >> 16) <= clen && t.x + (t.w & 0xffffu) <= L;
        }
        if (!uni((uint32_t)fits)) {
            if (lane == 0) ntok[r] = nt | kTokBad;
            continue;
        }
        // one segment: its entry, its lane entry, its position-index blocks
        auto put = [&](uint32_t k, uint32_t x, uint32_t ex, uint32_t kz, uint32_t w) {
            const bool plain = (kz >> 30) == 0;
            if (seg) put_ent(seg, k, mk4(x, ex, kz, w));
            if (lanes) {
                const int64_t d = (int64_t)comp_addr - (int64_t)(uint64_t)(lanes + k);
                *(PX_GAS u32x4 *)(lanes + k) = mk4(x | ex << 16, kz, w, plain ? (uint32_t)(int32_t)(d >> 3) : (uint32_t)kRelNone);
            }
            if (pidx_n)
                for (uint32_t b = (x + 15) >> 4, b1 = min((ex + 15) >> 4, pidx_n); b < b1; ++b) pidx[b] = (uint16_t)k;
        };
        uint32_t ns = 0, px = 0, po = 0;  // segments so far; doc position and comp offset after the last token
        for (uint32_t i0 = 0; i0 < nt; i0 += 64) {
            const uint32_t i = i0 + lane;
            const bool in = i < nt;
            u32x4 tv = mk4(0, 0, 0, 0);
            if (in) tv = *(const PX_GAS u32x4 *)(tk + i);
            const TokEnt t{tv.x, tv.y, tv.z, tv.w};
            const uint32_t rl = t.rs & 0xffffu, sz = t.rs >> 16;
            // the doc position and comp offset after the previous token
            uint32_t ex_prev = (uint32_t)__shfl_up((int)(t.x + rl), 1), eo_prev = (uint32_t)__shfl_up((int)(t.o + sz), 1);
            if (lane == 0) {
                ex_prev = px;
                eo_prev = po;
            }
            const bool plain = in && t.o > eo_prev;
            const uint32_t c = in ? (plain ? 2u : 1u) : 0u;
            uint32_t incl = c;
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)incl, o);
                if (lane >= o) incl += y;
            }
            const uint32_t k0 = ns + incl - c;
            if (plain) put(k0, ex_prev, t.x, eo_prev, 0u);
            if (in) put(k0 + (plain ? 1u : 0u), t.x, t.x + rl, t.o | kSegRecord, t.w);
            const uint32_t last = min(nt - i0, 64u) - 1u;
            ns += (uint32_t)__shfl((int)incl, (int)last);
            px = (uint32_t)__shfl((int)(t.x + rl), (int)last);
            po = (uint32_t)__shfl((int)(t.o + sz), (int)last);
        }
        if (lane == 0) {
            if (po < clen) put(ns++, px, L, po, 0u);  // the doc's last plain bytes
            if (seg) put_ent(seg, ns, mk4(L, L, clen | kSegEnd, 0));
            if (lanes) *(PX_GAS u32x4 *)(lanes + ns) = mk4(L | L << 16, clen | kSegEnd, 0, 0);
        }
        ns = uni(readlane(ns, 0));
        // blocks past the source end: no segment
        if (pidx_n)
            for (uint32_t b = (L + 15) / 16 + lane; b < pidx_n; b += 64) pidx[b] = (uint16_t)min(ns, 65535u);
        // lane entries need 16-bit coordinates and a comp base within +-16 GiB (k_tokenize's rule)
        bool mono = true;
        if (lanes) {
            const int64_t d0 = (int64_t)comp_addr - (int64_t)(uint64_t)lanes,
                          d1 = (int64_t)comp_addr - (int64_t)(uint64_t)(lanes + ns);
            mono = mono && (d0 >> 3) == (int64_t)(int32_t)(d0 >> 3) && (d1 >> 3) == (int64_t)(int32_t)(d1 >> 3);
        }
        if (lane == 0) {
            nseg_out[r] = ns | (mono && pidx_n ? 0u : kNoPidx);
            // (no lane entries and no segment entries: nothing could decode it -- cannot happen)
            status[r] = !seg && !(mono && pidx_n && lanes) ? kErrCorrupt : kOk;
        }
    }
}

// 48-byte records moved as three 16-byte vectors (struct copies cannot cross address spaces)
template <class T>
PX_DEV T load48(const PX_GAS T *p) {
    static_assert(sizeof(T) == 48, "48-byte record");
    const PX_GAS u32x4 *v = (const PX_GAS u32x4 *)p;
    u32x4 w[3] = {v[0], v[1], v[2]};
    T t;
    __builtin_memcpy(&t, w, 48);
    return t;
}
template <class T>
PX_DEV void store48(PX_GAS T *p, const T &t) {
    u32x4 w[3];
    __builtin_memcpy(w, &t, 48);
    PX_GAS u32x4 *v = (PX_GAS u32x4 *)p;
    v[0] = w[0];
    v[1] = w[1];
    v[2] = w[2];
}

struct SlotV {
    const PX_GAS uint8_t *comp;
    const PX_GAS u32x4 *seg;  // entry k: seg[k] = {x, ex, kz, aux}
    const PX_GAS uint16_t *pidx;
    const PX_GAS u32x4 *lane;  // LaneEnt k = lane[k] (null: serial decode only)
    uint32_t nseg, pidx_n;
};

PX_DEV SlotV slot_at(const PX_GAS RecSlot *slots, uint32_t r) {
    const RecSlot s = load48(slots + r);
    SlotV v;
    v.comp = (const PX_GAS uint8_t *)s.comp;
    v.seg = (const PX_GAS u32x4 *)s.seg;
    v.pidx = (const PX_GAS uint16_t *)s.pidx;
    v.lane = (const PX_GAS u32x4 *)s.lane;
    v.nseg = s.nseg;
    v.pidx_n = s.pidx_n;
    return v;
}
PX_DEV SlotV slot_uniform(const PX_GAS RecSlot *slots, uint32_t r) {
    SlotV v = slot_at(slots, r);
    v.comp = (const PX_GAS uint8_t *)uni64((uint64_t)v.comp);
    v.seg = (const PX_GAS u32x4 *)uni64((uint64_t)v.seg);
    v.pidx = (const PX_GAS uint16_t *)uni64((uint64_t)v.pidx);
    v.lane = (const PX_GAS u32x4 *)uni64((uint64_t)v.lane);
    v.nseg = uni(v.nseg);
    v.pidx_n = uni(v.pidx_n);
    return v;
}

// Segment entry k as {x, ex, kz, aux}.  A record built from the encoder's tokens keeps only
// its lane entries (16-bit x / ex, the same kz / aux): its seg pointer is null.  A record
// parsed by k_tokenize (source positions may wrap: 32-bit x) keeps both.
PX_DEV u32x4 seg_ent(const PX_GAS u32x4 *seg, const PX_GAS u32x4 *lane, uint32_t k) {
    if (seg) return seg[k];
    const u32x4 l = lane[k];
    return mk4(l.x & 0xffffu, l.x >> 16, l.y, l.z);
}
PX_DEV u32x4 seg_ent(const SlotV &s, uint32_t k) { return seg_ent(s.seg, s.lane, k); }

// Resolve every record token of the new records to the entry of its target record
// that holds the token's `from` (the decoder's lanes then walk entries by address).
__global__ void __launch_bounds__(256) k_link(uint32_t n, const LinkJob *jobs) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t j = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); j < n; j += waves) {
        const LinkJob job = jobs[j];
        PX_GAS u32x4 *seg = (PX_GAS u32x4 *)job.seg;
        PX_GAS u32x4 *lanes = (PX_GAS u32x4 *)job.lane;
        const PX_GAS RecSlot *slots = (const PX_GAS RecSlot *)job.slots;
        if (!lanes) continue;
        for (uint32_t k = lane; k < job.nseg; k += 64) {
            const u32x4 e = seg_ent(seg, lanes, k);
            if ((e.z >> 30) != 2) continue;
            const uint32_t ridx = e.w & 0xffffu, rfrom = e.w >> 16;
            int32_t rel = kRelNone;
            if (ridx < job.nrec) {
                const SlotV t = slot_at(slots, ridx);
                if (t.pidx_n && (rfrom >> 4) < t.pidx_n && t.lane) {
                    uint32_t k2 = min((uint32_t)t.pidx[rfrom >> 4], t.nseg);
                    while (k2 < t.nseg && seg_ent(t, k2).y <= rfrom) ++k2;
                    const int64_t d = ((int64_t)(uint64_t)(t.lane + k2) - (int64_t)(uint64_t)(lanes + k)) / 16;
                    if (d > INT32_MIN && d <= INT32_MAX) rel = (int32_t)d;
                }
            }
            lanes[k].w = (uint32_t)rel;
        }
    }
}

// ====================================================================== decode
// One wave per query.  A frame (the reference's PXSGen over one record range) is
// consumed 64 segments at a time: lane l takes segment f.seg + l, a prefix scan of
// the requested sizes gives every lane its ret cursor and its output offset, and
// each lane expands its own record reference depth-first, walking the linked
// segment entries by address with a small per-lane stack in LDS (deeper frames
// spill to the wave's free serial frames) and writing straight to the output.  A
// lane whose work leaves the simple case (a periodic self reference, nesting past
// the spill, an output that would reach the consumer's cap or
// exceed what it asked for, an unlinked token) ends the batch; that one segment
// then goes through the serial frame machine (a stack of Frames in scratch memory),
// which is the reference's generator nesting restated.
#ifndef PX_LANE_DEPTH
#define PX_LANE_DEPTH 4
#endif
#ifndef PX_DEC_WAVES
#define PX_DEC_WAVES 4
#endif
constexpr uint32_t kLaneDepth = PX_LANE_DEPTH;  // 4: 4 KB of LDS per wave; registers then bound occupancy (28 waves/CU)
#ifndef PX_LANE_SPILL
#define PX_LANE_SPILL 32
#endif
constexpr uint32_t kLaneSpill = PX_LANE_SPILL;  // lane frames past kLaneDepth, in scratch memory
constexpr uint32_t kLaneCopyMax = 512;  // plain pieces up to this size are copied by one lane
constexpr uint32_t kAssignMin = 24;      // idle lanes that trigger an assignment round

// Copies use unaligned 16-byte accesses (gfx950 runs in unaligned access mode; the
// compiler itself emits them for byte-aligned memcpy).  Sources are compressed
// bytes, destinations the query output: they never overlap.
typedef uint32_t u32x4_u __attribute__((ext_vector_type(4), aligned(1)));
PX_DEV u32x4 ld16(const PX_GAS uint8_t *p) { return *(const PX_GAS u32x4_u *)p; }
PX_DEV void st16(PX_GAS uint8_t *p, u32x4 v) { *(PX_GAS u32x4_u *)p = v; }
PX_DEV void copy16(PX_GAS uint8_t *dst, const PX_GAS uint8_t *src) { st16(dst, ld16(src)); }

PX_DEV void wave_copy(PX_GAS uint8_t *dst, const PX_GAS uint8_t *src, uint32_t n) {
    const uint32_t l16 = lane_id() * 16;
    uint32_t o = 0;
    for (; o + 4096 <= n; o += 4096) {  // four 16-byte loads in flight per lane
        const u32x4 v0 = ld16(src + o + l16), v1 = ld16(src + o + 1024 + l16), v2 = ld16(src + o + 2048 + l16),
                    v3 = ld16(src + o + 3072 + l16);
        st16(dst + o + l16, v0);
        st16(dst + o + 1024 + l16, v1);
        st16(dst + o + 2048 + l16, v2);
        st16(dst + o + 3072 + l16, v3);
    }
    for (; o + 1024 <= n; o += 1024) copy16(dst + o + l16, src + o + l16);
    const uint32_t full = (n - o) / 16;
    if (l16 < full * 16) copy16(dst + o + l16, src + o + l16);
    const uint32_t t = o + full * 16 + lane_id();
    if (t < n) dst[t] = src[t];
}

// one lane copies its own n bytes.  Every load is issued before the first store
// (source and destination never overlap, but the compiler cannot know that), so a
// piece of up to 64 bytes costs one memory round trip, not one per 16 bytes.
PX_DEV void lane_copy(PX_GAS uint8_t *dst, const PX_GAS uint8_t *src, uint32_t n) {
    if (n >= 16 && n <= 32) {
        const u32x4 v0 = ld16(src), v1 = ld16(src + n - 16);
        st16(dst, v0);
        st16(dst + n - 16, v1);
        return;
    }
    if (n > 32 && n <= 64) {
        const uint32_t o1 = 16u, o2 = min(32u, n - 16), o3 = n - 16;
        const u32x4 v0 = ld16(src), v1 = ld16(src + o1), v2 = ld16(src + o2), v3 = ld16(src + o3);
        st16(dst, v0);
        st16(dst + o1, v1);
        st16(dst + o2, v2);
        st16(dst + o3, v3);
        return;
    }
    if (n >= 16) {
        uint32_t i = 0;
        for (; i + 64 <= n; i += 64) {
            const u32x4 v0 = ld16(src + i), v1 = ld16(src + i + 16), v2 = ld16(src + i + 32), v3 = ld16(src + i + 48);
            st16(dst + i, v0);
            st16(dst + i + 16, v1);
            st16(dst + i + 32, v2);
            st16(dst + i + 48, v3);
        }
        for (; i + 16 <= n; i += 16) copy16(dst + i, src + i);
        if (i < n) copy16(dst + n - 16, src + n - 16);  // overlapping tail, same bytes
        return;
    }
    if (n >= 8) {
        uint64_t a, b;
        __builtin_memcpy(&a, (const PX_GAS void *)src, 8);
        __builtin_memcpy(&b, (const PX_GAS void *)(src + n - 8), 8);
        __builtin_memcpy((PX_GAS void *)dst, &a, 8);
        __builtin_memcpy((PX_GAS void *)(dst + n - 8), &b, 8);
        return;
    }
    if (n >= 4) {
        uint32_t a, b;
        __builtin_memcpy(&a, (const PX_GAS void *)src, 4);
        __builtin_memcpy(&b, (const PX_GAS void *)(src + n - 4), 4);
        __builtin_memcpy((PX_GAS void *)dst, &a, 4);
        __builtin_memcpy((PX_GAS void *)(dst + n - 4), &b, 4);
        return;
    }
    if (n) {  // 1..3 bytes: first, middle, last (loads first)
        const uint8_t a = src[0], b = src[n >> 1], c = src[n - 1];
        dst[0] = a;
        dst[n >> 1] = b;
        dst[n - 1] = c;
    }
}

// the first r < 16 bytes of v to dst: one predicated store per set bit of r (8, 4, 2,
// 1 bytes), the same four store instructions for every lane whatever its r
PX_DEV uint32_t dw_at(u32x4 v, uint32_t i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
PX_DEV void st_tail(PX_GAS uint8_t *dst, u32x4 v, uint32_t r) {
    if (r & 8) {
        const uint64_t x = ((uint64_t)v.y << 32) | v.x;
        __builtin_memcpy((PX_GAS void *)dst, &x, 8);
    }
    const uint32_t o8 = r & 8, o4 = r & 12, o2 = r & 14;
    if (r & 4) {
        const uint32_t x = dw_at(v, o8 >> 2);
        __builtin_memcpy((PX_GAS void *)(dst + o8), &x, 4);
    }
    if (r & 2) {
        const uint16_t x = (uint16_t)dw_at(v, o4 >> 2);
        __builtin_memcpy((PX_GAS void *)(dst + o4), &x, 2);
    }
    if (r & 1) dst[o2] = (uint8_t)(dw_at(v, o2 >> 2) >> (8 * (o2 & 3)));
}
// one lane copies a piece of n bytes.  Below 64 bytes: the 16-byte blocks and the tail
// block are loaded together (the tail load may read up to 15 bytes past the piece: every
// source is compressed bytes with >= 64 bytes of slack behind them in its store), then
// stored, so a wave of mixed piece sizes issues at most 4 loads and 7 stores instead of
// one load/store pair per size class.  Longer pieces take lane_copy.
PX_DEV void span_copy(PX_GAS uint8_t *dst, const PX_GAS uint8_t *src, uint32_t n) {
    if (n >= 64) {
        lane_copy(dst, src, n);
        return;
    }
    const uint32_t f = n & ~15u;
    const u32x4 t = ld16(src + f);
    u32x4 a0{}, a1{}, a2{};
    if (f >= 16) a0 = ld16(src);
    if (f >= 32) a1 = ld16(src + 16);
    if (f >= 48) a2 = ld16(src + 32);
    if (f >= 16) st16(dst, a0);
    if (f >= 32) st16(dst + 16, a1);
    if (f >= 48) st16(dst + 32, a2);
    st_tail(dst + f, t, n & 15);
}

PX_DEV int32_t wave_excl_scan(int32_t v) {
    int32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        int32_t y = __shfl_up(x, o);
        if ((int)lane_id() >= o) x += y;
    }
    return x - v;
}

// length of the run of 251 bytes ending at comp[ci], not looking below comp[lo]
PX_DEV uint32_t esc_run_lane(const PX_GAS uint8_t *comp, uint32_t lo, uint32_t ci) {
    uint32_t run = 0;
    while (run <= ci - lo && comp[ci - run] == kEsc) ++run;
    return run;
}
PX_DEV uint32_t esc_run_wave(const PX_GAS uint8_t *comp, uint32_t lo, uint32_t ci) {
    const uint32_t lane = lane_id();
    uint32_t run = 0;
    for (;;) {
        uint32_t top = ci + 1 - run;  // scan [top-64, top)
        uint32_t span = min(64u, top - lo);
        bool is_e = lane < span && comp[top - 1 - lane] == kEsc;
        uint64_t nm = ballot(lane < span && !is_e);
        if (nm) return run + ffs64(nm);
        run += span;
        if (span < 64) return run;
    }
}

// first segment of s whose end is beyond `from` (wave-uniform)
PX_DEV uint32_t seg_find(const SlotV &s, int32_t from) {
    const uint32_t lane = lane_id();
    uint32_t lo = 0, hi = s.nseg;  // answer in [lo, hi]
    if (s.pidx_n && from >= 0 && ((uint32_t)from >> 4) < s.pidx_n) {
        lo = min((uint32_t)uni(s.pidx[(uint32_t)from >> 4]), hi);
        for (;;) {  // at most 16 source bytes past a segment start: one probe, almost always
            uint32_t k = lo + lane;
            uint64_t m = ballot(k < hi && (int32_t)seg_ent(s, k).y > from);
            if (m) return lo + ffs64(m);
            if (hi - lo <= 64) return hi;
            lo += 64;
        }
    }
    while (hi - lo > 64) {
        uint32_t step = (hi - lo + 63) / 64;
        uint32_t k = lo + lane * step;
        bool le = k < hi && (int32_t)seg_ent(s, k).y <= from;  // segment k ends at or before from
        uint64_t m = ballot(le);
        uint32_t cnt = (uint32_t)__popcll(m);  // prefix of lanes with le (monotone)
        uint32_t nlo = cnt ? lo + (cnt - 1) * step + 1 : lo;
        uint32_t nhi = min(hi, lo + cnt * step);
        lo = uni(nlo);
        hi = uni(nhi);
    }
    uint32_t k = lo + lane;
    bool le = k < hi && (int32_t)seg_ent(s, k).y <= from;
    return uni(lo + (uint32_t)__popcll(ballot(le)));
}

// Output writers of the decoder.  Byte output (getitem) copies bytes; address output
// (k_decode_addr, the span build) writes, at the first output byte of each run copied from
// consecutive compressed bytes, the address of its first source byte relative to the query
// record's comp pointer (kAddrNone for a run reaching beyond +-2 GiB of it); the run's other
// bytes keep the kAddrMark the array was filled with.  (One store per run: a lane writing its
// run's addresses byte by byte was most of the span build's decode.)
PX_DEV int32_t addr_of(const PX_GAS uint8_t *p, const PX_GAS uint8_t *qb) {
    const int64_t d = (int64_t)((uint64_t)p - (uint64_t)qb);
    return (d == (int64_t)(int32_t)d && (int32_t)d != kAddrNone && (int32_t)d != kAddrMark) ? (int32_t)d : kAddrNone;
}
PX_DEV int32_t run_addr(const PX_GAS uint8_t *p, uint32_t n, const PX_GAS uint8_t *qb) {
    const int32_t a = addr_of(p, qb);
    return a != kAddrNone && addr_of(p + (n - 1), qb) != kAddrNone ? a : kAddrNone;
}
PX_DEV void out_wave_copy(PX_GAS uint8_t *dst, const PX_GAS uint8_t *src, uint32_t n, const PX_GAS uint8_t *) {
    wave_copy(dst, src, n);
}
PX_DEV void out_wave_copy(PX_GAS int32_t *dst, const PX_GAS uint8_t *src, uint32_t n, const PX_GAS uint8_t *qb) {
    if (n && lane_id() == 0) dst[0] = run_addr(src, n, qb);
}
PX_DEV void out_lane_copy(PX_GAS uint8_t *dst, const PX_GAS uint8_t *src, uint32_t n, const PX_GAS uint8_t *) {
    lane_copy(dst, src, n);
}
PX_DEV void out_lane_copy(PX_GAS int32_t *dst, const PX_GAS uint8_t *src, uint32_t n, const PX_GAS uint8_t *qb) {
    if (n) dst[0] = run_addr(src, n, qb);
}
PX_DEV void out_one(PX_GAS uint8_t *dst, const PX_GAS uint8_t *src, const PX_GAS uint8_t *) { *dst = *src; }
PX_DEV void out_one(PX_GAS int32_t *dst, const PX_GAS uint8_t *src, const PX_GAS uint8_t *qb) {
    *dst = addr_of(src, qb);
}
// A window stopped by a short or flagged segment redoes its output from `from`; address output
// clears the run starts its abandoned lanes left in [from, to) (the redo may cut runs elsewhere)
PX_DEV void out_clear(PX_GAS uint8_t *, uint32_t, uint32_t) {}
PX_DEV void out_clear(PX_GAS int32_t *o, uint32_t from, uint32_t to) {
    __threadfence_block();
    for (uint32_t i = from + lane_id(); i < to; i += 64) o[i] = kAddrMark;
    __threadfence_block();
}
// A periodic record token repeats its child's output [s, s + produced) to end (PiXiuStr.h:168-181).
// Address output first writes every address of the child's output (the repeat copies them by
// position); its first byte is a run start.
PX_DEV void out_repeat(PX_GAS uint8_t *o, uint32_t s, uint32_t produced, uint32_t end) {
    for (uint32_t k = produced + lane_id(); s + k < end; k += 64) o[s + k] = o[s + (k % produced)];
}
PX_DEV void out_repeat(PX_GAS int32_t *o, uint32_t s, uint32_t produced, uint32_t end) {
    const uint32_t lane = lane_id();
    int32_t carry = kAddrNone;  // the address of the byte before the window
    for (uint32_t i0 = 0; i0 < produced; i0 += 64) {
        const uint32_t i = i0 + lane;
        const bool in = i < produced;
        const int32_t raw = in ? o[s + i] : kAddrMark;
        const uint64_t sm = ballot(in && raw != kAddrMark);
        const uint64_t le = sm & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));  // starts at or below the lane
        const uint32_t sl = le ? 63u - (uint32_t)__clzll((long long)le) : 0u;
        const int32_t sv = (int32_t)__shfl(raw, (int)sl);
        const int32_t base = le ? sv : carry;
        const int32_t dist = le ? (int32_t)(lane - sl) : (int32_t)lane + 1;
        const int32_t v = base == kAddrNone ? kAddrNone : base + dist;
        if (in && raw == kAddrMark) o[s + i] = v;
        carry = (int32_t)__shfl(v, (int)(min(produced - i0, 64u) - 1u));
    }
    __threadfence_block();
    for (uint32_t k = produced + lane; s + k < end; k += 64) o[s + k] = o[s + (k % produced)];
}

struct DecLds {
    // per-lane frames, 4 words: entry address | rec << 48, from | len << 16, ret
    uint32_t stk[kLaneDepth * 4][64];
};

constexpr uint32_t kDecWaves = PX_DEC_WAVES;  // independent query waves per block (see kGstWaves)

// the body of k_decode (getitem queries) and k_decode_keys (the stored-key prefixes
// setitem and prefix iteration decode): one code, two kernel names in the profiles
template <class OutT>
PX_DEV void decode_body(const DecodeQuery *qs, uint32_t nq, const RecSlot *const *chunk_slots, OutT *out_,
                        uint32_t *out_len, uint32_t *status, Frame *scratch, uint32_t depth_cap,
                        uint32_t n_waves) {
    __shared__ DecLds lds_w[kDecWaves];
    const uint32_t wv = uni(threadIdx.x >> 6);
    // bit 31: XCD-aware order.  Blocks are dealt round-robin over the 8 XCDs (b and
    // b + 8 share one); with the remap, XCD x takes a contiguous range of queries
    // (the host sorts them by chunk), so each chunk's compressed bytes and entries are
    // read through one XCD's L2 instead of all eight
    uint32_t lb = blockIdx.x;
    if (n_waves >> 31) {
        const uint32_t nb = gridDim.x, x = blockIdx.x & 7u, per = nb >> 3, rem = nb & 7u;
        lb = x * per + min(x, rem) + (blockIdx.x >> 3);
    }
    n_waves &= 0x7fffffffu;
    const uint32_t gw = lb * kDecWaves + wv;
    if (gw >= n_waves) return;
    DecLds &lds = lds_w[wv];
    const uint32_t lane = lane_id();
    PX_GAS Frame *stk = (PX_GAS Frame *)scratch + (size_t)gw * depth_cap;
#ifdef PX_PROFILE
    uint64_t prof[P_N] = {};
    const uint64_t t_kernel0 = __builtin_amdgcn_s_memtime();
#endif
    for (uint32_t qi = gw; qi < nq; qi += n_waves) {
        const DecodeQuery q = qs[qi];
        const uint32_t qchunk = uni(q.chunk);
        const PX_GAS RecSlot *slots = qchunk == kNone ? nullptr : (const PX_GAS RecSlot *)chunk_slots[qchunk];
        const bool compat = uni(q.mode) == 0;
        const uint32_t nrec = uni(q.nrec);
        PX_GAS OutT *o = (PX_GAS OutT *)out_ + uni64(q.out_off);
        const PX_GAS uint8_t *qb =
            slots && uni(q.idx) < nrec ? (const PX_GAS uint8_t *)uni64((uint64_t)slot_at(slots, uni(q.idx)).comp) : nullptr;
        const uint32_t qcap = uni(q.out_cap);
        // the top frame's ret cursor in record coordinates: a piece [from, to) of a compat drain
        // cut at token starts continues the whole drain's cursor (the self-overlap test of a
        // record token compares against it, PiXiuStr.h:163-170)
        const int32_t qbase = unii((int32_t)q.pad);
        uint32_t outp = 0, err = 0, depth = 0;
        bool capped = false;

        auto push = [&](uint32_t r, int32_t from, int32_t to, uint32_t cap) -> bool {
            if (r >= nrec) {
                err = kErrCorrupt;  // PiXiuChunk::getitem past the chunk (the oracle's ECORRUPT)
                return false;
            }
            if (depth >= depth_cap) {
                err = kErrDepth;
                return false;
            }
            const SlotV sv = slot_uniform(slots, r);
            Frame f;
            f.rec = r;
            f.from = from;
            f.len = to - from;
            f.ret = 0;
            f.src = 0;
            f.seg = sv.nseg ? seg_find(sv, from) : 0;
            f.cap = cap;
            f.state = 0;
            f.pstart = 0;
            f.sub_from = f.sub_to = f.supply = 0;
            store48(stk + depth, f);
            ++depth;
            return true;
        };

        // Consume frame f's segments with dynamic lane assignment: every idle lane
        // takes the next unassigned segment (in order), so a lane that finishes a
        // short expansion picks up new work instead of waiting for the slowest lane
        // of a fixed 64-segment batch.  Output offsets and ret cursors come from
        // running prefix sums of the requested sizes (a wave scan per assignment
        // round).  A segment that leaves the lane path (flag) or produces fewer bytes
        // than it requested (short) sets `stop`: segments before it are committed,
        // later ones are abandoned and redone.  Returns true when the segment at
        // f.seg must go through the serial path next.
        auto window = [&](Frame &f, const SlotV &sv) -> bool {
            if (!sv.lane) return true;  // no lane entries: the serial path takes every segment
            const int32_t rbase = depth == 1 ? qbase : 0;
            // lane frames past the LDS stack spill to this wave's unused serial frames
            // (stk[depth, depth_cap) are free while the window runs): 1 KB per level
            PX_GAS u32x4 *spill = (PX_GAS u32x4 *)(stk + depth);
            const uint32_t dmax = kLaneDepth + min(kLaneSpill, (depth_cap - depth) * 3u / 64u);
            const uint32_t outp0 = outp;
            const int32_t ret0 = f.ret;
            uint32_t next = f.seg;     // next unassigned segment
            uint32_t end = sv.nseg;    // shrinks to the first inactive segment
            int32_t run_req = ret0;    // ret cursor at `next`
            uint32_t run_out = outp0;  // output position at `next`
            // stop key = 2 * (first segment not committed) + (0: it goes serial, 1: it does not)
            uint32_t stop_key = 0xffffffffu, stop_out = 0;
            int32_t stop_ret = 0;
            // prefetched lane entries of segments [next, next + 64): lane l holds next + l
            u32x4 PE = mk4(0, 0, 0, 0);
            {
                const uint32_t kk = next + lane;
                if (kk < end) PE = sv.lane[kk];
            }
            // per-lane segment state
            uint32_t k = kNone, base = 0, w = 0, wmax = 0;
            int32_t kret = 0;
            bool busy = false, flag = false, pmode = false, fresh = false;
            const PX_GAS uint8_t *psrc = nullptr;
#ifdef PX_PROFILE
            uint32_t freason = 0, freason_first = 0;
            uint32_t lane_it = 0, nspill = 0;  // (nspill: this lane's frames stored past the LDS stack)
#endif
            // walk state
            const PX_GAS u32x4 *e = nullptr;  // the lane entry F was loaded from
            u32x4 F = mk4(0, 0, 0, 0);
            uint32_t rec = 0, d = 0;
            int32_t from = 0, len = 0, ret = 0;
            PX_CNT(P_D_BATCH, 1);
#ifdef PX_PROFILE
            const uint64_t t_lane0 = __builtin_amdgcn_s_memtime();
#endif
            for (;;) {
                const uint32_t lim = min(end, stop_key >> 1);
                const uint64_t im = ballot(k == kNone);
                // an assignment round once enough lanes are idle (or none is working)
                if (next < lim && im && (__popcll(im) >= kAssignMin || !ballot(busy))) {
#ifdef PX_PROFILE
                    const uint64_t t_as0 = __builtin_amdgcn_s_memtime();
#endif
                    // ---- assignment round: idle lane of rank r takes segment next + r
                    const uint32_t rank =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(im >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)im, 0));
                    const bool take = k == kNone && next + rank < lim;
                    const int src_l = (int)(rank & 63u);
                    const u32x4 E = mk4(__shfl(PE.x, src_l), __shfl(PE.y, src_l), __shfl(PE.z, src_l),
                                        __shfl(PE.w, src_l));
                    const int32_t sx = (int32_t)(E.x & 0xffffu), ex = (int32_t)(E.x >> 16);
                    const uint32_t kind = E.y >> 30, cs = E.y & kSegMask;
                    const uint32_t ridx = E.z & 0xffffu;
                    const int32_t rfrom = (int32_t)(E.z >> 16), supply = ex - sx, rto = rfrom + supply;
                    const int32_t p0 = max(sx, f.from);
                    const int32_t sub_from = rfrom + max(0, f.from - sx);
                    const bool enter = kind == 2 && sx - 1 + supply >= f.from;
                    int32_t req = 0;
                    if (take && kind == 0 && p0 < ex) req = ex - p0;
                    if (take && enter) req = rto - sub_from;
                    const int32_t ret_l = run_req + wave_incl_scan_dpp(req) - req;
                    const bool active = take && ret_l < f.len;  // a prefix of the takers
                    const int32_t need = f.len - ret_l;
                    int32_t reqc = 0, sub_to = 0;
                    uint32_t csrc = 0;
                    bool child = false, fl = false;
                    if (active && kind == 0 && p0 < ex) {
                        const int32_t avail = ex - p0;
                        reqc = min(avail, need);
                        csrc = cs + (uint32_t)(p0 - sx);
                        // the range ends here: if its last byte opens a 251 pair, the pair
                        // is written whole (per-token length check, PiXiuStr.h:136,142-147)
                        if (avail > need && compat && (esc_run_lane(sv.comp, cs, csrc + (uint32_t)reqc - 1) & 1))
                            ++reqc;
                    } else if (active && enter) {
                        sub_to = min(rto, sub_from + need);
                        const int32_t stp = compat ? ret_l + rbase : max(sx, f.from);
                        if (ridx >= nrec || (sub_from < stp && stp < sub_to && ridx == f.rec)) {
                            fl = true;
                            PX_FR(1);
                        }
                        reqc = sub_to - sub_from;
                        child = true;
                    }
                    // every active segment before the last one asks for exactly req bytes, so
                    // the output offset follows the same scan
                    const uint32_t b = run_out + (uint32_t)(ret_l - run_req);
                    if (active && (uint64_t)b + (uint64_t)reqc >= f.cap) {
                        fl = true;
                        PX_FR(2);
                    }
                    const uint64_t am = ballot(active);
                    const uint32_t na = (uint32_t)__popcll(am), nt = (uint32_t)__popcll(ballot(take));
                    if (na) {
                        const uint32_t hl = 63u - (uint32_t)__clzll((long long)am);  // highest active lane
                        run_req = unii(readlane((uint32_t)(ret_l + req), hl));
                        run_out = uni(readlane(b + (uint32_t)reqc, hl));
                    }
                    if (na < nt) end = next + na;  // the frame's range ends inside this round
                    next += na;
                    if (active) {
                        k = next - na + rank;
                        base = b;
                        kret = ret_l;
                        wmax = (uint32_t)reqc;
                        w = 0;
                        flag = fl;
                    }
                    // long plain pieces: copied by the whole wave now; shorter ones by their
                    // lane, 64 bytes per walk step
                    uint64_t lm = ballot(active && !fl && kind == 0 && reqc > (int32_t)kLaneCopyMax);
                    while (lm) {
                        const uint32_t j = ffs64(lm);
                        lm &= lm - 1;
                        out_wave_copy(o + readlane(b, j), sv.comp + readlane(csrc, j), readlane((uint32_t)reqc, j), qb);
                    }
                    if (active && !fl && kind == 0 && reqc > 0 && reqc <= (int32_t)kLaneCopyMax) {
                        // a shorter plain piece: copied by its lane in the walk steps below,
                        // where its loads overlap the walking lanes' loads
                        busy = true;
                        pmode = true;
                        psrc = sv.comp + csrc;
                    } else if (active && !fl && !child) {
                        w = (uint32_t)reqc;
                        k = kNone;  // done (a plain or empty segment is never short)
                    }
                    if (active && !fl && child) {
                        e = (int32_t)E.w == kRelNone ? nullptr : sv.lane + (next - na + rank) + (int32_t)E.w;
                        if (!e) {
                            PX_FR(3);
                            flag = true;  // token without a linked target
                        } else {
                            // the first entry is loaded by the lane's first walk step
                            busy = true;
                            fresh = true;
                            rec = ridx;
                            d = 0;
                            from = sub_from;
                            len = reqc;
                            ret = 0;
                        }
                    }
                    // refill the prefetch buffer from the new `next`
                    {
                        const uint32_t kk = next + lane;
                        if (kk < end) PE = sv.lane[kk];
                    }
#ifdef PX_PROFILE
                    prof[P_D_T_ASSIGN] += __builtin_amdgcn_s_memtime() - t_as0;
                    prof[P_D_ROUNDS] += 1;
#endif
                }
                // ---- one walk step for every busy lane
                bool done = false;
                if (ballot(busy)) {
                    PX_CNT(P_D_LANEIT, 1);
#ifdef PX_PROFILE
                    lane_it += 1;
#endif
                    if (busy) {
                        const int32_t x = (int32_t)(F.x & 0xffffu), y = (int32_t)(F.x >> 16);
                        const uint32_t kd = F.y >> 30;
                        const PX_GAS u32x4 *ne = fresh ? e : e + 1;
                        uint32_t nb = 0, poff = 0;
                        bool ov = false;
                        // a plain entry's first comp byte: the record's comp base (rel, in 8-byte
                        // units from the entry) + the segment's comp offset
                        const PX_GAS uint8_t *seg0 =
                            (const PX_GAS uint8_t *)e + (int64_t)(int32_t)F.w * 8 + (F.y & kSegMask);
                        if (pmode) {
                            seg0 = psrc;
                            nb = min(wmax - w, 64u);
                            psrc += nb;
                            if (w + nb == wmax) {
                                pmode = false;
                                busy = false;
                                done = true;
                            }
                        } else if (fresh) {
                            fresh = false;  // this step only loads the first entry
                        } else if (ret >= len || kd == 3) {
                            if (d == 0) {
                                busy = false;
                                done = true;
                            } else {
                                --d;
                                u32x4 W;
                                if (d < kLaneDepth)
                                    W = mk4(lds.stk[d * 4 + 0][lane], lds.stk[d * 4 + 1][lane], lds.stk[d * 4 + 2][lane],
                                            lds.stk[d * 4 + 3][lane]);
                                else
                                    W = spill[(d - kLaneDepth) * 64 + lane];
                                ne = (const PX_GAS u32x4 *)((uint64_t)W.x | (uint64_t)(W.y & 0xffffu) << 32);
                                rec = W.y >> 16;
                                from = (int32_t)(W.z & 0xffffu);
                                len = (int32_t)(W.z >> 16);
                                ret = (int32_t)W.w;
                            }
                        } else if (kd == 0) {
                            const int32_t q0 = max(x, from);
                            if (q0 < y) {
                                const int32_t avail = y - q0, nd = len - ret;
                                const uint32_t n = (uint32_t)min(avail, nd);
                                if (w + n > wmax) {
                                    PX_FR(4);
                                    flag = true;
                                    busy = false;
                                } else {
                                    nb = n;
                                    poff = (uint32_t)(q0 - x);
                                    ov = avail > nd && compat;
                                }
                            }
                        } else if (kd == 2) {
                            const int32_t sup = y - x;
                            if (x - 1 + sup >= from) {
                                const uint32_t ri = F.z & 0xffffu;
                                const int32_t rf = (int32_t)(F.z >> 16), rt = rf + sup;
                                const int32_t sf = rf + max(0, from - x);
                                const int32_t st = min(rt, sf + (len - ret));
                                const int32_t stp = compat ? ret : max(x, from);
                                const PX_GAS u32x4 *t = (int32_t)F.w == kRelNone ? nullptr : e + (int32_t)F.w;
                                const uint64_t nx = (uint64_t)(e + 1);
                                if (!t || ri >= nrec || (ri == rec && sf < stp && stp < st) || d + 1 >= dmax ||
                                    (uint32_t)from > 0xffffu || (uint32_t)len > 0xffffu || (nx >> 48) != 0) {
                                    PX_FR(!t ? 3 : ri >= nrec ? 8 : (ri == rec && sf < stp && stp < st) ? 5 : d + 1 >= dmax ? 6 : 7);
                                    flag = true;  // leaves the lane path: serial machine
                                    busy = false;
                                } else {
                                    const u32x4 W = mk4((uint32_t)nx, (uint32_t)(nx >> 32) | rec << 16,
                                                        (uint32_t)from | (uint32_t)len << 16, (uint32_t)(ret + (st - sf)));
                                    if (d < kLaneDepth) {
                                        lds.stk[d * 4 + 0][lane] = W.x;
                                        lds.stk[d * 4 + 1][lane] = W.y;
                                        lds.stk[d * 4 + 2][lane] = W.z;
                                        lds.stk[d * 4 + 3][lane] = W.w;
                                    } else {
                                        spill[(d - kLaneDepth) * 64 + lane] = W;
#ifdef PX_PROFILE
                                        ++nspill;
#endif
                                    }
                                    ++d;
                                    ne = t;  // the target's entry holding rf; entries before sf are passed over
                                    rec = ri;
                                    from = sf;
                                    len = st - sf;
                                    ret = 0;
                                }
                            }
                        }
                        // next entry first (every entry a lane can reach is in bounds: a
                        // record's entries end with a sentinel, which pops)
                        u32x4 NF = F;
                        if (busy && !pmode) NF = ne[0];
                        if (nb) {
                            const PX_GAS uint8_t *cp = seg0 + poff;
                            const uint32_t last = ov ? cp[nb - 1] : 0u;
                            out_lane_copy(o + base + w, cp, nb, qb);
                            w += nb;
                            ret += (int32_t)nb;
                            // a range ending inside a 251 pair writes the pair whole
                            if (last == kEsc && (esc_run_lane(seg0, 0, poff + nb - 1) & 1)) {
                                if (w + 1 > wmax) {
                                    PX_FR(4);
                                    flag = true;
                                    busy = false;
                                } else {
                                    out_one(o + base + w, cp + nb, qb);
                                    ++w;
                                    ++ret;
                                }
                            }
                        }
                        F = NF;
                        e = ne;
                    }
                }
                // ---- events: a flagged segment (goes serial) or a short one (committed,
                // but later offsets are wrong) moves `stop` down
                const bool fl_ev = k != kNone && flag;
                const bool sh_ev = k != kNone && done && w != wmax;
                if (ballot(fl_ev || sh_ev)) {
                    uint32_t key = fl_ev ? 2u * k : sh_ev ? 2u * (k + 1u) + 1u : 0xffffffffu;
                    uint32_t mn = key;
                    for (int ofs = 32; ofs >= 1; ofs >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, ofs));
                    mn = uni(mn);
                    if (mn < stop_key) {
                        const uint32_t hl = ffs64(ballot((fl_ev || sh_ev) && key == mn));
                        stop_key = mn;
                        if (mn & 1u) {  // short: committed through it
                            stop_out = uni(readlane(base + w, hl));
                            stop_ret = unii(readlane((uint32_t)kret + wmax, hl));
                        } else {
#ifdef PX_PROFILE
                            freason_first = readlane(freason, hl);
#endif
                            stop_out = uni(readlane(base, hl));
                            stop_ret = unii(readlane((uint32_t)kret, hl));
                        }
                    }
                }
                if (done) k = kNone;
                // abandon flagged lanes and everything at or past stop
                if (k != kNone && (flag || k >= (stop_key >> 1))) {
                    k = kNone;
                    busy = false;
                    pmode = false;
                    fresh = false;
                }
                flag = flag && k != kNone;
#ifdef PX_PROFILE
                if (k == kNone) freason = 0;
#endif
                if (!ballot(k != kNone) && next >= min(end, stop_key >> 1)) break;
            }
#ifdef PX_PROFILE
            prof[P_D_T_LANE] += __builtin_amdgcn_s_memtime() - t_lane0;
            for (int ofs = 32; ofs >= 1; ofs >>= 1) nspill += (uint32_t)__shfl_xor((int)nspill, ofs);
            prof[P_D_SPILL] += nspill;
            {
                uint32_t mx = lane_it;
                prof[P_D_MAXIT] += uni(mx);
            }
#endif
            if (stop_key != 0xffffffffu && (stop_key >> 1) <= next) {
                PX_CNT(P_D_COMMIT, (stop_key >> 1) - f.seg);
                out_clear(o, stop_out, run_out);
                f.seg = stop_key >> 1;
                outp = stop_out;
                f.ret = stop_ret;
                const bool serial = (stop_key & 1u) == 0;
#ifdef PX_PROFILE
                if (serial) prof[P_DF_NONE + freason_first] += 1;
                PX_CNT(P_D_FLAGGED, serial ? 1 : 0);
                PX_CNT(P_D_SHORT, serial ? 0 : 1);
#endif
                return serial;
            }
            PX_CNT(P_D_COMMIT, next - f.seg);
            f.seg = next;
            f.ret = ret0 + (int32_t)(run_out - outp0);
            outp = run_out;
            return false;
        };

        if (qchunk == kNone || !push(uni(q.idx), unii(q.from), unii(q.to), qcap)) {
            if (lane == 0) {
                out_len[qi] = 0;
                status[qi] = err ? err : kErrInval;
            }
            continue;
        }
        while (depth > 0 && !err) {
            __builtin_amdgcn_wave_barrier();
            Frame f = load48(stk + (depth - 1));
            f.rec = uni(f.rec);
            f.from = unii(f.from);
            f.len = unii(f.len);
            f.ret = unii(f.ret);
            f.seg = uni(f.seg);
            f.cap = uni(f.cap);
            f.state = uni(f.state);
            f.pstart = uni(f.pstart);
            f.sub_from = unii(f.sub_from);
            f.sub_to = unii(f.sub_to);
            f.supply = unii(f.supply);
            const SlotV sv = slot_uniform(slots, f.rec);
            const int32_t rbase = depth == 1 ? qbase : 0;
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
                            out_repeat(o, f.pstart, produced, end);
                            outp = end;
                            if (outp >= f.cap) pop = true;
                        }
                    }
                    if (!pop) {
                        f.ret += f.sub_to - f.sub_from;
                        ++f.seg;
                        f.state = 0;
                    }
                }
            }
            bool pushed = false;
            while (!pop && !pushed && !err && f.ret < f.len && f.seg < sv.nseg) {
                if (!window(f, sv)) continue;
                PX_CNT(P_D_SERIAL, 1);
                // one segment through the serial machine
                const u32x4 E = seg_ent(sv, f.seg);
                const int32_t sx = (int32_t)uni(E.x), ex = (int32_t)uni(E.y);
                const uint32_t sz = uni(E.z), sw = uni(E.w);
                const uint32_t cs = sz & kSegMask;
                if ((sz >> 30) == 2) {
                    const int32_t ridx = (int32_t)(sw & 0xffffu);
                    const int32_t rfrom = (int32_t)(sw >> 16);
                    const int32_t supply = ex - sx;
                    const int32_t rto = rfrom + supply;
                    if (sx - 1 + supply >= f.from) {
                        int32_t sub_from = rfrom + max(0, f.from - sx);
                        int32_t sub_to = min(rto, sub_from + (f.len - f.ret));
                        int32_t stop = compat ? f.ret + rbase : max(sx, f.from);
                        bool periodic = sub_from < stop && stop < sub_to && (uint32_t)ridx == f.rec;
                        f.state = periodic ? 2 : 1;
                        f.pstart = outp;
                        f.sub_from = sub_from;
                        f.sub_to = sub_to;
                        f.supply = supply;
                        __builtin_amdgcn_wave_barrier();
                        store48(stk + (depth - 1), f);
                        uint32_t ccap = periodic ? min(f.cap, outp + (uint32_t)(sub_to - sub_from)) : f.cap;
                        bool ok = periodic ? push(f.rec, sub_from, stop, ccap) : push((uint32_t)ridx, sub_from, sub_to, ccap);
                        if (!ok) break;
                        PX_CNT(P_D_PUSH, 1);
                        pushed = true;
                        break;
                    }
                    ++f.seg;
                } else if ((sz >> 30) == 1) {
                    ++f.seg;
                } else {
                    const int32_t p0 = max(sx, f.from);
                    if (p0 < ex) {
                        uint32_t avail = (uint32_t)(ex - p0);
                        uint32_t need = (uint32_t)(f.len - f.ret);
                        uint32_t nb = min(avail, need);
                        if (avail > need && compat) {
                            uint32_t ci = cs + (uint32_t)(p0 - sx) + nb - 1;
                            if (esc_run_wave(sv.comp, cs, ci) & 1) nb += 1;
                        }
                        uint32_t room = f.cap > outp ? f.cap - outp : 0;
                        uint32_t w = min(nb, room);
                        out_wave_copy(o + outp, sv.comp + cs + (uint32_t)(p0 - sx), w, qb);
                        outp += w;
                        f.ret += (int32_t)nb;
                        if (w < nb || outp >= f.cap) {
                            pop = true;
                            break;
                        }
                    }
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
#ifdef PX_PROFILE
    prof[P_D_T_TOTAL] = __builtin_amdgcn_s_memtime() - t_kernel0;
    if (lane == 0)
        for (int k = P_D_BATCH; k < P_N; ++k) atomicAdd(&g_prof[k], (unsigned long long)prof[k]);
#endif
}

__global__ void __launch_bounds__(64 * kDecWaves) k_decode(const DecodeQuery *qs, uint32_t nq,
                                                         const RecSlot *const *chunk_slots, uint8_t *out,
                                                         uint32_t *out_len, uint32_t *status, Frame *scratch,
                                                         uint32_t depth_cap, uint32_t n_waves) {
    decode_body(qs, nq, chunk_slots, out, out_len, status, scratch, depth_cap, n_waves);
}
__global__ void __launch_bounds__(64 * kDecWaves) k_decode_keys(const DecodeQuery *qs, uint32_t nq,
                                                              const RecSlot *const *chunk_slots, uint8_t *out,
                                                              uint32_t *out_len, uint32_t *status, Frame *scratch,
                                                              uint32_t depth_cap, uint32_t n_waves) {
    decode_body(qs, nq, chunk_slots, out, out_len, status, scratch, depth_cap, n_waves);
}
// the same decode with address output (span build; out_off counts 4-byte elements)
__global__ void __launch_bounds__(64 * kDecWaves) k_decode_addr(const DecodeQuery *qs, uint32_t nq,
                                                              const RecSlot *const *chunk_slots, int32_t *out,
                                                              uint32_t *out_len, uint32_t *status, Frame *scratch,
                                                              uint32_t depth_cap, uint32_t n_waves) {
    decode_body(qs, nq, chunk_slots, out, out_len, status, scratch, depth_cap, n_waves);
}

// ====================================================================== spans
// Span build: one wave per record scans its address decode (run starts, kAddrMark between:
// each byte's address is expanded from its run's start).  A span starts where the address is
// not the previous one + 1.  Count pass: spans (| kSpanBad for a source out
// of the relative range, | kSpanEq when the expansion equals the doc, i.e. compat ==
// exact).  Write pass: {rel, start} entries plus the {0, len} sentinel.
#ifndef PX_SPAN_STEPS
#define PX_SPAN_STEPS 8
#endif
constexpr uint32_t kSpanSteps = PX_SPAN_STEPS;
PX_DEV void span_job(const SpanJob &jb) {
    const uint32_t lane = lane_id();
    const PX_GAS uint8_t *base = (const PX_GAS uint8_t *)jb.base;
    const PX_GAS uint8_t *doc = (const PX_GAS uint8_t *)jb.doc;
    PX_GAS SpanEnt *out = (PX_GAS SpanEnt *)jb.out;
    const uint32_t len = uni(jb.len);
    uint32_t cnt = 0;
    bool bad = false, eq = doc && len == uni(jb.doc_len);
    int32_t prev_last = kAddrNone;  // address of the byte before k0 (lane 63 of the last step)
    // pieces: output bytes [o, o + pn) of the record are at a (a piece's bytes are contiguous)
    const uint32_t np = jb.pq ? uni(jb.last) - uni(jb.first) : 1u;
    uint32_t o = 0;
    for (uint32_t pi = 0; pi < np; ++pi) {
        const PX_GAS int32_t *a = (const PX_GAS int32_t *)jb.addr;
        uint32_t pn = len;
        if (jb.pq) {
            const uint32_t j = uni(jb.first) + pi;
            a += uni64(jb.pq[j].out_off);
            pn = min(uni(jb.pl[j]), len - o);
        }
        // kSpanSteps 64-byte steps per group: their address loads, then their doc / comp byte
        // loads for the compat == exact test, each issued together (one wave walks a record:
        // its dependent loads were the pass's time; 8 steps in flight instead of 4, round 6)
        for (uint32_t g0 = 0; g0 < pn; g0 += 64u * kSpanSteps) {
            int32_t raw[kSpanSteps], vv[kSpanSteps];
#pragma unroll
            for (uint32_t u = 0; u < kSpanSteps; ++u) {
                const uint32_t i = g0 + 64u * u + lane;
                raw[u] = i < pn ? a[i] : kAddrMark;
            }
#pragma unroll
            for (uint32_t u = 0; u < kSpanSteps; ++u) {
                const uint32_t i0 = g0 + 64u * u;
                vv[u] = kAddrNone;
                if (i0 >= pn) break;  // (wave-uniform)
                const uint32_t i = i0 + lane, k = o + i;
                const bool in = i < pn;
                // the byte's address: its run's start address + its distance from the start (the
                // latest start at or below the lane, else the previous window's last address + 1)
                const uint64_t le = ballot(in && raw[u] != kAddrMark) & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
                const uint32_t sl = le ? 63u - (uint32_t)__clzll((long long)le) : 0u;
                const int32_t sv = (int32_t)__shfl(raw[u], (int)sl);
                const int32_t rb = le ? sv : prev_last;
                const int32_t v = !in ? 0 : rb == kAddrNone ? kAddrNone : rb + (le ? (int32_t)(lane - sl) : (int32_t)lane + 1);
                vv[u] = in ? v : kAddrNone;
                int32_t pv = __shfl_up(v, 1);
                if (lane == 0) pv = prev_last;
                const bool start = in && (k == 0 || pv == kAddrNone || v != pv + 1);
                bad = bad || (bool)ballot(in && v == kAddrNone);
                const uint64_t m = ballot(start);
                if (out && !bad) {
                    const uint32_t rank =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
                    if (start) {
                        PX_GAS uint32_t *e = (PX_GAS uint32_t *)(out + cnt + rank);
                        e[0] = (uint32_t)v;
                        e[1] = k;
                    }
                    // tile index: the span holding byte k, at every tile start
                    if (jb.tix && in && (k % kGatherTile) == 0)
                        ((PX_GAS uint32_t *)jb.tix)[k / kGatherTile] = cnt + rank + (start ? 1u : 0u) - 1u;
                }
                cnt += (uint32_t)__popcll(m);
                const uint32_t nl = min(pn - i0, 64u);  // (the piece's last byte of this step)
                prev_last = __shfl(v, (int)(nl - 1));
            }
            if (eq) {
                uint32_t bb[kSpanSteps], dd[kSpanSteps];
#pragma unroll
                for (uint32_t u = 0; u < kSpanSteps; ++u) {
                    const uint32_t i = g0 + 64u * u + lane;
                    const bool ok = i < pn && vv[u] != kAddrNone;
                    bb[u] = ok ? base[vv[u]] : 0u;
                    dd[u] = ok ? doc[o + i] : 0u;
                }
                bool mis = false;
#pragma unroll
                for (uint32_t u = 0; u < kSpanSteps; ++u) {
                    const uint32_t i = g0 + 64u * u + lane;
                    mis = mis || (i < pn && (vv[u] == kAddrNone || bb[u] != dd[u]));
                }
                eq = !ballot(mis);
            }
        }
        o += pn;
    }
    if (out && !bad && lane == 0) {
        PX_GAS uint32_t *e = (PX_GAS uint32_t *)(out + cnt);
        e[0] = 0;
        e[1] = len;
    }
    if (!out && lane == 0) jb.count[0] = cnt | (bad ? kSpanBad : 0u) | (eq ? kSpanEq : 0u);
}

// The span build's jobs straight from the address decode's own queries and results (no job
// table from the host): job j is query j (chunk-ordered), its addresses at out_off, its
// compressed bytes from the chunk's slot table, its doc from src[j].  Count pass (tab null):
// cnt[j] = spans | kSpanBad | kSpanEq (kSpanBad also for a failed decode), ents[j] = its
// entries with the sentinel, tiles[j] = its tile-index words (both 0 without a table).
// Write pass: the table and tile index at the inclusive scans' offsets.
__global__ void __launch_bounds__(256) k_span_jobs(uint32_t n, const DecodeQuery *dq, const uint32_t *dl,
                                                   const uint32_t *ds, const SpanSrc *src,
                                                   const RecSlot *const *chunk_slots, const int32_t *addr,
                                                   uint32_t *cnt, uint32_t *ents, uint32_t *tiles,
                                                   const uint32_t *eoff_incl, const uint32_t *toff_incl, SpanEnt *tab,
                                                   uint32_t *tixb, const DecodeQuery *pq, const uint32_t *pl,
                                                   const uint32_t *pfirst) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t j = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); j < n; j += waves) {
        const DecodeQuery &q = dq[j];
        const uint32_t st = uni(ds[j]), len = uni(dl[j]);
        SpanJob jb;
        jb.addr = pq ? addr : addr + q.out_off;
        jb.pq = pq;
        jb.pl = pl;
        jb.first = pq ? pfirst[j] : 0u;
        jb.last = pq ? pfirst[j + 1] : 0u;
        jb.base = chunk_slots[uni(q.chunk)][uni(q.idx)].comp;
        jb.doc = src[j].doc;
        jb.len = len;
        jb.doc_len = uni(src[j].doc_len);
        jb.count = cnt + j;
        jb.out = nullptr;
        jb.tix = nullptr;
        if (!tab) {
            if (st != kOk) {
                if (lane == 0) {
                    cnt[j] = kSpanBad;
                    ents[j] = 0;
                    tiles[j] = 0;
                }
                continue;
            }
            span_job(jb);
            if (lane == 0) {
                const uint32_t c = cnt[j];
                const bool ok = !(c & kSpanBad);
                ents[j] = ok ? (c & ~(kSpanBad | kSpanEq)) + 1u : 0u;
                tiles[j] = ok ? (len + kGatherTile - 1) / kGatherTile : 0u;
            }
        } else {
            if (uni(cnt[j]) & kSpanBad) continue;
            jb.out = tab + (eoff_incl[j] - ents[j]);
            jb.tix = tixb + (toff_incl[j] - tiles[j]);
            span_job(jb);
        }
    }
}

// Gather: a full-range getitem served from its span table.  One wave per task of 64
// consecutive tiles of the launch; lane j assembles tile g0 + j: kGatherTile (32) output
// bytes of one query, two 16-byte blocks.  Its first span comes from the tile index; spans
// come in seven at a time (eight 8-byte entries: the eighth start ends the seventh span).
// Every load of a batch is issued before any is used -- the pieces' source loads do not sit
// behind one another's latency: the seven spans' first pieces (each up to its 16-byte block's
// end) and the continuation of the span that crosses the block boundary.  Each piece is read
// with one unaligned 16-byte load, shifted to its byte offset and merged into its block; the
// tile leaves with two aligned 16-byte stores.  Queries are 16-byte aligned in the output
// and own >= 64 bytes past their expansion (out_cap = doc + 64, rounded to 16), so whole
// 16-byte blocks are stored; sources have >= 64 bytes of slack behind them; reads of entries
// past a table's sentinel stay inside the table allocation (its tile index and 64-byte tail
// follow) and are never used.
PX_DEV u32x4 shl_bytes(u32x4 w, uint32_t b) {  // byte i of the result = byte i - b of w (0 below)
    const uint32_t ds = b >> 2, bs = b & 3u;
    uint32_t t[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = i - (int)ds;
        t[i] = k == 0 ? w.x : k == 1 ? w.y : k == 2 ? w.z : k == 3 ? w.w : 0u;
    }
    if (bs == 0) return u32x4{t[0], t[1], t[2], t[3]};
    const uint32_t sh = 4u - bs;
    return u32x4{__builtin_amdgcn_alignbyte(t[0], 0u, sh), __builtin_amdgcn_alignbyte(t[1], t[0], sh),
                 __builtin_amdgcn_alignbyte(t[2], t[1], sh), __builtin_amdgcn_alignbyte(t[3], t[2], sh)};
}
PX_DEV uint32_t byte_mask(int lo, int hi) {  // bytes [lo, hi) of a dword (clamped to 0..4)
    lo = max(lo, 0);
    hi = min(hi, 4);
    if (hi <= lo) return 0u;
    const uint32_t m = hi - lo == 4 ? 0xffffffffu : ((1u << (8 * (hi - lo))) - 1u);
    return m << (8 * lo);
}
// v (output-aligned) masked to bytes [lo, hi) of a 16-byte block (empty when hi <= lo)
PX_DEV u32x4 mask_piece(u32x4 v, int lo, int hi) {
    return u32x4{v.x & byte_mask(lo, hi), v.y & byte_mask(lo - 4, hi - 4), v.z & byte_mask(lo - 8, hi - 8),
                 v.w & byte_mask(lo - 12, hi - 12)};
}

// the task table: per 64-tile task, its first query, the span holding the task's first tile
// in that query's table, and the tiles (bits) where later queries start.  One wave per query:
// a query owns the tasks whose first tile is one of its tiles (every task has exactly one
// owner, so nothing is zeroed and nothing is atomic); only its last owned task can hold the
// starts of later queries (tile0 rises strictly), found by one load per lane.  `ctl`
// (device-driven launches, px_keyidx.hip): skip everything unless no key missed and the
// output fits -- the task table is sized for that bound.
__global__ void __launch_bounds__(256) k_gather_tasks(uint32_t nq, const GatherQuery *qs, GatherTask *task,
                                                      const uint32_t *ctl, uint64_t out_cap) {
    const uint32_t q = uni(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)), lane = lane_id();
    if (q >= nq) return;
    if (ctl && (uni(ctl[0]) != 0u || (uint64_t)uni(ctl[1]) * 16u > out_cap)) return;
    const GatherQuery &Q = qs[q];
    const uint32_t len = uni(Q.len), tile0 = uni(Q.tile0);
    const uint32_t nt = max(1u, (min(len, uni(Q.cap)) + kGatherTile - 1) / kGatherTile);
    const uint32_t ntix = (len + kGatherTile - 1) / kGatherTile;  // (the tile index's length)
    const uint32_t T0 = (tile0 + 63u) >> 6, T1 = (tile0 + nt - 1u) >> 6;
    if (T0 > T1) return;  // (the query lies inside a task owned by an earlier one)
    unsigned long long M = 0;
    {
        const uint32_t j = q + 1u + lane;
        if (j < nq) {
            const uint32_t t0 = qs[j].tile0;
            if (t0 < 64u * (T1 + 1u)) M = 1ull << (t0 - 64u * T1);
        }
#pragma unroll
        for (int o = 32; o; o >>= 1) M |= __shfl_xor(M, o);
    }
    const uint32_t *tix = Q.tix;
    for (uint32_t T = T0 + lane; T <= T1; T += 64) {
        const uint32_t g = 64u * T - tile0;
        GatherTask d;
        d.q0 = q;
        d.k0 = g < ntix ? tix[g] : 0u;
        d.M = T == T1 ? M : 0ull;
        task[T] = d;
    }
}

// Gather (see the comment above shl_bytes): one wave per task of 64 tiles.  The TA (the
// per-CU address unit) bounds this kernel -- every lane of a scattered 16-byte load is an
// address of its own (rocprofv3: TA_BUSY ~70 % of the launch, r03w) -- so the wave keeps
// vector loads to the ones that carry bytes: its first query comes in by scalar loads
// (every lane of a wave that lies in one query), the span entries of that query from the
// task's first tile on are staged in LDS by two coalesced loads per lane and each lane finds
// its own span there, and a source load is issued only by the lanes whose span has a piece.
#ifndef PX_GATHER_STAGE
#define PX_GATHER_STAGE 256
#endif
constexpr uint32_t kGatherStage = PX_GATHER_STAGE;
PX_DEV void gather_task(uint32_t ti, const GatherTask *task, const GatherQuery *qs, uint32_t nq, uint8_t *out_,
                        uint32_t *out_len, uint32_t *status, uint2 *stage, uint8_t *tl) {
    const uint32_t lane = lane_id();
    const uint32_t g0 = ti * 64, q0 = uni(task[ti].q0), k0 = uni(task[ti].k0);
    const uint64_t M = ((uint64_t)uni((uint32_t)(task[ti].M >> 32)) << 32) | uni((uint32_t)task[ti].M);
    const uint32_t qi = q0 + (uint32_t)__popcll(M & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull)));
    // the first query, by scalar loads (uniform address)
    const GatherQuery &Q0 = qs[q0];
    const PX_GAS uint2 *sp0 = (const PX_GAS uint2 *)Q0.span;
    const uint32_t nent0 = uni(Q0.nspan) + 1u;  // (the sentinel included)
    const uint32_t nst = min(kGatherStage, nent0 > k0 ? nent0 - k0 : 0u);
    // its entries [k0, k0 + nst): coalesced, two entries per lane per load
    {
        u32x4 sv[kGatherStage / 128];
#pragma unroll
        for (uint32_t r = 0; r < kGatherStage / 128; ++r) {  // (both loads out before either is stored)
            const uint32_t j = r * 128 + 2 * lane;
            if (j + 1 < nst) {
                sv[r] = *(const PX_GAS u32x4_u *)(sp0 + k0 + j);
            } else if (j < nst) {
                sv[r] = u32x4{sp0[k0 + j].x, sp0[k0 + j].y, 0u, 0u};
            }
        }
#pragma unroll
        for (uint32_t r = 0; r < kGatherStage / 128; ++r) {
            const uint32_t j = r * 128 + 2 * lane;
            if (j < nst) stage[j] = uint2{sv[r].x, sv[r].y};
            if (j + 1 < nst) stage[j + 1] = uint2{sv[r].z, sv[r].w};
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (qi >= nq) return;
    const bool fast = qi == q0;
    GatherQuery q;
    if (M == 0) {  // (uniform) every lane in the first query
        q = Q0;
    } else {
        q = qs[qi];
    }
    const uint32_t t = g0 + lane - q.tile0;
    const uint32_t lim = min(q.len, q.cap), a = t * kGatherTile;
    if (t == 0) {
        out_len[q.slot] = lim;
        status[q.slot] = q.len > q.cap ? (uint32_t)kErrSpace : (uint32_t)kOk;
    }
    if (a >= lim) return;
    const uint32_t e = min(a + kGatherTile, lim), B = a + 16;  // B: the second block's first byte
    const PX_GAS uint8_t *base = (const PX_GAS uint8_t *)q.base;
    const PX_GAS uint32_t *sp = (const PX_GAS uint32_t *)q.span;  // {rel, start} pairs, then the sentinel
    // the span holding byte a: the last staged entry starting at or before a (the staged
    // range starts with the span holding the task's first tile); the tile index otherwise
    uint32_t k;
    if (fast && nst && stage[nst - 1].y > a) {
        uint32_t lo = 0, hi = nst - 1;  // stage[lo].y <= a < stage[hi].y
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (stage[mid].y <= a) lo = mid;
            else hi = mid;
        }
        k = k0 + lo;
    } else {
        k = ((const PX_GAS uint32_t *)q.tix)[t];
    }
    // the tile is assembled in LDS: each span piece is written whole (16 unaligned bytes from
    // its first source byte, at its output offset), in output order, so the bytes a write puts
    // past its piece are overwritten by the pieces after it (the last one's land in the pad)
    for (;;) {
        uint32_t en[16];
        if (fast && k - k0 + 8 <= nst) {  // (staged)
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const uint2 x = stage[k - k0 + v];
                en[2 * v] = x.x;
                en[2 * v + 1] = x.y;
            }
        } else {
#pragma unroll
            for (int v = 0; v < 4; ++v) *(u32x4 *)(en + 4 * v) = *(const PX_GAS u32x4_u *)(sp + 2 * k + 4 * v);
        }
        // span h covers output [st_h, st_{h+1}); alive while no earlier start reached e (the
        // sentinel's start is the length: entries past it are never used).  A piece is at most
        // 32 bytes, and at most one piece of a 32-byte tile is longer than 16 (its second half
        // is one more load).
        uint32_t live = 0;  // bit h: span h has a piece in the tile (an unbroken run from bit 0)
        bool alive = true;
        int32_t off[7];
        uint32_t d0[7];
        uint32_t lh = 7;  // the piece longer than 16 bytes (7: none)
#pragma unroll
        for (int h = 0; h < 7; ++h) {
            const uint32_t st = en[2 * h + 1], nx = en[2 * h + 3];
            const uint32_t x0 = max(st, a), x1 = min(nx, e);
            alive = alive && st < e;  // (then x0 < x1: span 0 holds byte a, later ones start past it)
            off[h] = alive ? (int32_t)en[2 * h] + (int32_t)(x0 - st) : 0;
            d0[h] = x0 - a;
            live |= alive ? 1u << h : 0u;
            if (alive && x1 - x0 > 16) lh = h;
        }
        // every load of the batch goes out before any is used, each from the lanes that need it
        u32x4 v[7];
        u32x4 vl = {0, 0, 0, 0};
#pragma unroll
        for (int h = 0; h < 7; ++h) {
            v[h] = u32x4{0, 0, 0, 0};
            if ((live >> h) & 1u) v[h] = ld16(base + off[h]);
        }
        const int32_t loff = lh < 7 ? off[lh < 7 ? lh : 0] + 16 : 0;
        if (lh < 7) vl = ld16(base + loff);
#pragma unroll
        for (int h = 0; h < 7; ++h) {
            if (!((live >> h) & 1u)) continue;
            *(u32x4_u *)(tl + d0[h]) = v[h];
            if (lh == (uint32_t)h) *(u32x4_u *)(tl + d0[h] + 16) = vl;
        }
        // done once span k + 7 starts past the tile, or the sentinel came
        if (live != 0x7fu || en[15] >= e) break;
        k += 7;
    }
    u32x4 r0 = *(const u32x4 *)tl, r1 = *(const u32x4 *)(tl + 16);
    if (e - a < kGatherTile) {  // the record's last tile: zeros past its end, as before
        r0 = mask_piece(r0, 0, (int)(e - a));
        r1 = mask_piece(r1, 0, (int)(e - a) - 16);
    }
    PX_GAS uint8_t *o = (PX_GAS uint8_t *)out_ + q.out_off + a;
    *(PX_GAS u32x4 *)o = r0;
    if (B < e) *(PX_GAS u32x4 *)(o + 16) = r1;
}

// One wave per task.  The tasks are cut into eight contiguous ranges, one per XCD
// (blockIdx.x & 7: neighbouring tasks read neighbouring span tables and chunks through the
// same L2); the waves of an XCD's range go out in task order.  `ctl` (device-driven
// launches): the grid is sized for an upper bound on the tasks, the real count comes from
// the device (waves past it exit at once), with the same skip as k_gather_tasks.
__global__ void __launch_bounds__(256) k_gather(uint32_t ntask_h, const uint32_t *ctl, uint64_t out_cap,
                                                const GatherTask *task, const GatherQuery *qs, uint32_t nq,
                                                uint8_t *out_, uint32_t *out_len, uint32_t *status) {
    __shared__ uint2 stage_all[4][kGatherStage];
    __shared__ u32x4 tile_all[4][64 * 3];  // per lane: its 32-byte tile and a 16-byte pad
    uint32_t ntask = ntask_h;
    if (ctl) {
        if (uni(ctl[0]) != 0u || (uint64_t)uni(ctl[1]) * 16u > out_cap) return;
        ntask = (uni(ctl[2]) + 63u) / 64u;
    }
    const uint32_t w = threadIdx.x >> 6, per = (ntask + 7u) / 8u;
    const uint32_t j = (blockIdx.x >> 3) * (blockDim.x >> 6) + w;  // (the wave's place in its XCD's range)
    if (j >= per) return;
    const uint32_t ti = uni((blockIdx.x & 7u) * per + j);
    if (ti >= ntask) return;
    gather_task(ti, task, qs, nq, out_, out_len, status, stage_all[w], (uint8_t *)&tile_all[w][lane_id() * 3]);
}

// ====================================================================== migrate
// Re-insert the live-epoch entries of a child map into a larger (zeroed) table.
__global__ void __launch_bounds__(256) k_rehash(const uint4 *old_tab, uint32_t old_n, uint32_t epoch,
                                                uint4 *new_tab, uint32_t new_mask) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= old_n) return;
    uint4 e = old_tab[i];
    if ((e.x >> 26) != epoch) return;
    uint32_t parent = e.x & kNodeMask;
    uint32_t c = (e.w >> 16) & 0xffu;
    uint32_t nb = (new_mask + 1) / kBucket;
    uint32_t b = hslot(parent, c) & (nb - 1);
    for (;;) {
        for (uint32_t l = 0; l < kBucket; ++l) {
            uint32_t *slot = reinterpret_cast<uint32_t *>(&new_tab[b * kBucket + l]);
            if (atomicCAS(slot, 0u, e.x) == 0u) {
                slot[1] = e.y;
                slot[2] = e.z;
                slot[3] = e.w;
                return;
            }
        }
        b = (b + 1) & (nb - 1);
    }
}

}  // namespace

// ---------------------------------------------------------------------- launchers
namespace px {

hipError_t launch_doc_len(hipStream_t s, uint32_t n, const uint8_t *keys, const uint64_t *koff,
                          const uint8_t *vals, const uint64_t *voff, uint32_t *doc_len, uint32_t *rec_init) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_doc_len<<<blocks, 256, 0, s>>>(n, keys, koff, vals, voff, doc_len, rec_init);
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
                             uint8_t *const *comp_dst, const uint8_t *comp_base, uint32_t *msgs,
                             uint32_t *rec_chunk, uint32_t *rec_idx, uint32_t *rec_status, ShardState *st_out,
                             uint32_t *sink) {
    if (!n_shards) return hipSuccess;
    k_gst_encode<<<(n_shards + kGstWaves - 1) / kGstWaves, 64 * kGstWaves, 0, s>>>(
        shards, n_shards, doc_len, comp_dst, comp_base, msgs, rec_chunk, rec_idx, rec_status, st_out, sink);
    return hipGetLastError();
}

hipError_t launch_gst_emit(hipStream_t s, uint32_t n, const uint8_t *const *doc_ptr, const uint32_t *doc_len,
                           uint8_t *const *comp_dst, const uint8_t *comp_base, const uint32_t *msgs,
                           uint32_t *rec_status, uint32_t *comp_len, const uint64_t *tok_off, TokEnt *toks,
                           uint32_t *ntok) {
    if (!n) return hipSuccess;
    const uint32_t blocks = min((n + 3) / 4, 8192u);
    k_gst_emit<<<blocks, 256, 0, s>>>(n, doc_ptr, doc_len, comp_dst, comp_base, msgs, rec_status, comp_len, tok_off,
                                      toks, ntok);
    return hipGetLastError();
}

hipError_t launch_shard_init(hipStream_t s, uint32_t n, const ShardInit *jobs) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_shard_init<<<blocks, 256, 0, s>>>(n, jobs);
    return hipGetLastError();
}

hipError_t launch_scatter_slots(hipStream_t s, uint32_t n, const SlotPut *puts) {
    if (!n) return hipSuccess;
    k_scatter_slots<<<(n + 255) / 256, 256, 0, s>>>(n, puts);
    return hipGetLastError();
}

hipError_t launch_compact(hipStream_t s, uint32_t n, uint8_t *const *src, const uint32_t *len, uint8_t *dst,
                          const uint64_t *dst_off) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_compact<<<blocks, 256, 0, s>>>(n, src, len, dst, dst_off);
    return hipGetLastError();
}

hipError_t launch_count_esc(hipStream_t s, uint32_t n, uint8_t *const *src, const uint32_t *len, uint32_t *n_esc) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_count_esc<<<blocks, 256, 0, s>>>(n, src, len, n_esc);
    return hipGetLastError();
}

hipError_t launch_link(hipStream_t s, uint32_t n, const LinkJob *jobs) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_link<<<blocks, 256, 0, s>>>(n, jobs);
    return hipGetLastError();
}

hipError_t launch_tokenize(hipStream_t s, uint32_t n, const RecSlot *slots, uint32_t *nseg_out, uint32_t *status,
                           const uint32_t *ntok) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_tokenize<<<blocks, 256, 0, s>>>(n, slots, nseg_out, status, ntok);
    return hipGetLastError();
}
hipError_t launch_tok_segs(hipStream_t s, uint32_t n, const RecSlot *slots, const uint32_t *doc_len, const uint64_t *tok_off,
                           const TokEnt *toks, uint32_t *ntok, uint32_t *nseg_out, uint32_t *status) {
    if (!n) return hipSuccess;
    uint32_t blocks = min((n + 3) / 4, 8192u);
    k_tok_segs<<<blocks, 256, 0, s>>>(n, slots, doc_len, tok_off, toks, ntok, nseg_out, status);
    return hipGetLastError();
}

hipError_t launch_decode(hipStream_t s, const DecodeQuery *qs, uint32_t nq, const RecSlot *const *chunk_slots,
                         uint8_t *out, uint32_t *out_len, uint32_t *status, Frame *scratch, uint32_t depth_cap,
                         uint32_t n_waves, bool keys) {
    if (!nq) return hipSuccess;
    const uint32_t blocks = ((n_waves & 0x7fffffffu) + kDecWaves - 1) / kDecWaves;
    if (keys)
        k_decode_keys<<<blocks, 64 * kDecWaves, 0, s>>>(qs, nq, chunk_slots, out, out_len, status, scratch,
                                                          depth_cap, n_waves);
    else
        k_decode<<<blocks, 64 * kDecWaves, 0, s>>>(qs, nq, chunk_slots, out, out_len, status, scratch, depth_cap,
                                                     n_waves);
    return hipGetLastError();
}

hipError_t launch_decode_addr(hipStream_t s, const DecodeQuery *qs, uint32_t nq, const RecSlot *const *chunk_slots,
                              int32_t *out, uint32_t *out_len, uint32_t *status, Frame *scratch, uint32_t depth_cap,
                              uint32_t n_waves) {
    if (!nq) return hipSuccess;
    const uint32_t blocks = ((n_waves & 0x7fffffffu) + kDecWaves - 1) / kDecWaves;
    k_decode_addr<<<blocks, 64 * kDecWaves, 0, s>>>(qs, nq, chunk_slots, out, out_len, status, scratch, depth_cap,
                                                      n_waves);
    return hipGetLastError();
}

hipError_t launch_slot_place(hipStream_t s, uint32_t n, const RecSlot *src, const uint32_t *tok, const SlotDst *d,
                             LinkJob *jobs) {
    if (!n) return hipSuccess;
    k_slot_place<<<(n + 255) / 256, 256, 0, s>>>(n, src, tok, d, jobs);
    return hipGetLastError();
}
// A record decoded in pieces (the exact span build: exact parses of consecutive ranges are
// the consecutive slices of the doc): its length = the pieces' sum, its status = the first
// failing piece's.  first[k] .. first[k + 1] are record k's pieces.
// A record's pieces that reach its whole decode's room (cap) report kErrSpace, as the whole
// decode would.
__global__ void __launch_bounds__(256) k_span_agg(uint32_t n, const uint32_t *first, const uint32_t *pl,
                                                  const uint32_t *ps, const DecodeQuery *dq, uint32_t *dl, uint32_t *ds) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint64_t len = 0;
    uint32_t st = kOk;
    for (uint32_t j = first[k]; j < first[k + 1]; ++j) {
        len += pl[j];
        if (st == kOk) st = ps[j];
    }
    if (st == kOk && len >= dq[k].out_cap) st = kErrSpace;
    dl[k] = (uint32_t)min<uint64_t>(len, 0xffffffffu);
    ds[k] = st;
}
hipError_t launch_span_agg(hipStream_t s, uint32_t n, const uint32_t *first, const uint32_t *pl, const uint32_t *ps,
                           const DecodeQuery *dq, uint32_t *dl, uint32_t *ds) {
    if (!n) return hipSuccess;
    k_span_agg<<<(n + 255) / 256, 256, 0, s>>>(n, first, pl, ps, dq, dl, ds);
    return hipGetLastError();
}

// Compat pieces cut at token starts (build_spans): sub-query j is piece m of its record, nominal
// range [m * P, (m + 1) * P) of the record's source positions (from = m * P; out_off = the
// record's output base + 64 * m).  Its bounds move to the first token starting at or after
// each end (so a piece drains whole top-level tokens and the pieces' outputs, in order, are the
// whole drain's: PXSGen's ret cursor only counts requested bytes, PiXiuStr.h:136-192), its
// output to base + start + 64 * m with the piece's bytes + 64 of room, and `pad` carries the ret
// cursor at its start.  A record without a position index (source positions not monotone) or
// whose tokens cover more than its doc is drained whole by its piece 0.
__global__ void __launch_bounds__(256) k_span_pieces(uint32_t ns, DecodeQuery *sq, const RecSlot *const *chunk_slots,
                                                     uint32_t piece) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ns) return;
    DecodeQuery q = sq[j];
    const uint32_t m = (uint32_t)q.from / piece, L = q.pad;  // (pad: the record's doc length, on the way in)
    const uint64_t base = q.out_off - 64ull * m;
    const RecSlot *sl = chunk_slots[q.chunk] + q.idx;
    const uint32_t nseg = sl->nseg;
    const PX_GAS u32x4 *sg = (const PX_GAS u32x4 *)sl->seg, *ln = (const PX_GAS u32x4 *)sl->lane;
    auto seg_x = [&](uint32_t k) { return seg_ent(sg, ln, k).x; };
    auto seg_y = [&](uint32_t k) { return seg_ent(sg, ln, k).y; };
    const uint16_t *pidx = (const uint16_t *)sl->pidx;
    const uint32_t S = nseg && (sg || ln) ? seg_x(nseg) : 0u;  // (the end sentinel's position: the tokens' total)
    const bool split = nseg && sl->pidx_n && sl->lane && S <= L;
    auto bound = [&](uint32_t t) -> uint32_t {  // the first token start at or after t
        if (t == 0) return 0;
        if (t >= S) return S;
        uint32_t k = (t >> 4) < sl->pidx_n ? min((uint32_t)pidx[t >> 4], nseg) : nseg;
        while (k > 0 && seg_x(k) > t) --k;  // (a position index entry is the segment holding 16b)
        while (k < nseg && seg_y(k) <= t) ++k;
        return k >= nseg ? S : (seg_x(k) >= t ? seg_x(k) : seg_y(k));
    };
    if (!split) {
        q.from = 0;
        q.to = m == 0 ? (int32_t)kMaxDoc : 0;
        q.out_off = base;
        q.out_cap = m == 0 ? q.out_cap : 16u;  // (piece 0 keeps the whole record's room)
        q.pad = 0;
    } else {
        const uint32_t a = bound(m * piece), nominal_end = (m + 1) * piece;
        const bool last = nominal_end >= L;
        const uint32_t b = last ? S : bound(nominal_end);
        q.from = (int32_t)a;
        q.to = last ? (int32_t)kMaxDoc : (int32_t)b;
        q.out_off = base + a + 64ull * m;
        q.out_cap = b - a + 64u;
        q.pad = a;
    }
    sq[j] = q;
}
hipError_t launch_span_pieces(hipStream_t s, uint32_t ns, DecodeQuery *sq, const RecSlot *const *chunk_slots,
                              uint32_t piece) {
    if (!ns) return hipSuccess;
    k_span_pieces<<<(ns + 255) / 256, 256, 0, s>>>(ns, sq, chunk_slots, piece);
    return hipGetLastError();
}

hipError_t launch_span_jobs(hipStream_t s, uint32_t n, const DecodeQuery *dq, const uint32_t *dl, const uint32_t *ds,
                            const SpanSrc *src, const RecSlot *const *chunk_slots, const int32_t *addr, uint32_t *cnt,
                            uint32_t *ents, uint32_t *tiles, const uint32_t *eoff_incl, const uint32_t *toff_incl,
                            SpanEnt *tab, uint32_t *tixb, const DecodeQuery *pq, const uint32_t *pl,
                            const uint32_t *pfirst) {
    if (!n) return hipSuccess;
    k_span_jobs<<<std::min<uint32_t>((n + 3) / 4, 16384), 256, 0, s>>>(n, dq, dl, ds, src, chunk_slots, addr, cnt, ents,
                                                                       tiles, eoff_incl, toff_incl, tab, tixb, pq, pl,
                                                                       pfirst);
    return hipGetLastError();
}

// ntask: the tasks (ctl null), or (ctl: device-driven) an upper bound on them; task_buf holds
// gather_task_bytes(ntask)
uint64_t gather_task_bytes(uint32_t ntask) { return (uint64_t)ntask * sizeof(GatherTask) + 64; }
hipError_t launch_gather(hipStream_t s, uint32_t ntask, const uint32_t *ctl, uint64_t out_cap, void *task_buf,
                         const GatherQuery *qs, uint32_t nq, uint8_t *out, uint32_t *out_len, uint32_t *status) {
    if (!ntask || !nq) return hipSuccess;
    GatherTask *task = (GatherTask *)task_buf;
    k_gather_tasks<<<(nq + 3) / 4, 256, 0, s>>>(nq, qs, task, ctl, out_cap);
    // eight XCD ranges of ceil(ntask / 8) waves, 4 waves a workgroup
    const uint32_t grid = 8u * (((ntask + 7u) / 8u + 3u) / 4u);
    k_gather<<<grid, 256, 0, s>>>(ntask, ctl, out_cap, task, qs, nq, out, out_len, status);
    return hipGetLastError();
}

int debug_prof_take(unsigned long long *out, uint32_t cap) {
#ifdef PX_PROFILE
    uint32_t n = cap < (uint32_t)P_N ? cap : (uint32_t)P_N;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), n * 8) != hipSuccess) return -1;
    unsigned long long z[P_N] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z);
    return (int)n;
#else
    (void)out;
    (void)cap;
    return -1;
#endif
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

hipError_t launch_rehash(hipStream_t s, const uint4 *old_tab, uint32_t old_cap, uint32_t epoch,
                         uint4 *new_tab, uint32_t new_mask) {
    if (!old_cap) return hipSuccess;
    k_rehash<<<(old_cap + 255) / 256, 256, 0, s>>>(old_tab, old_cap, epoch, new_tab, new_mask);
    return hipGetLastError();
}

}  // namespace px
