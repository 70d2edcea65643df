// px_keyidx.hip — the device key index: getitem's key -> record resolution on the GPU.
//
// The CritBit stays the source of truth on the host (CritBitTree.cpp:180-196, 253-269).
// The index only mirrors the host's own fast path (px_runtime.cpp resolve_key): a raw key
// maps to the newest record stored under it, and that record answers the key when it is
// live and its compat-decoded key prefix is the escaped key -- exactly the record the
// CritBit walk reaches then.  Open addressing over 64-bit key hashes, verified against
// the raw key bytes; every key the index cannot answer sends the whole batch back to the
// host path, so results never depend on which path ran.
//
//   k_dk_insert   a set batch's new records (newest record id wins on a repeated key)
//   k_dk_kill     records the batch killed (replaces, deletes): live bit cleared
//   k_dk_lookup   one thread per query key: probe, verify, pick the span table; the batch's
//                 output offsets and first tiles in the same pass (a chained scan over the
//                 workgroups, decoupled look-back)
// The batch then goes straight to the gather (k_gather_tasks, k_gather) with no host round
// trip: ctl[0] = keys missed, ctl[1] = output bytes / 16, ctl[2] = tiles, ctl[3] = the
// index's insert-error word, ctl[4] = workgroup ticket, ctl[5] = queries past their room; both gather kernels skip the batch
// unless nothing missed and the output fits.
#include <hip/hip_runtime.h>

#include "px_common.h"

namespace px {
namespace {

#define DK_DEV __device__ __forceinline__

// keys are read 16 bytes at a time (unaligned loads), the bytes past a key's end masked off.
// The index's own key arena keeps >= 16 bytes of slack past its last key; a query key may sit
// at the very end of a caller's allocation (px_get_batch_dev reads the caller's device keys in
// place), so its last partial chunk is read byte by byte (SAFE) and nothing past it is touched.
#define DK_GAS __attribute__((address_space(1)))
typedef uint32_t dk_u4 __attribute__((ext_vector_type(4), aligned(1)));
DK_DEV uint32_t dk_word(const dk_u4 &v, int j, uint32_t left) {  // word j of v, bytes past `left` zeroed
    const uint32_t x = j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
    const uint32_t lo = 4u * (uint32_t)j;
    return left >= lo + 4u ? x : left <= lo ? 0u : x & ((1u << (8u * (left - lo))) - 1u);
}
template <bool SAFE>
DK_DEV dk_u4 dk_load(const DK_GAS uint8_t *p, uint32_t left) {
    if (!SAFE || left >= 16u) return *(const DK_GAS dk_u4 *)p;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t b = 0; b < left; ++b) w[b >> 2] |= (uint32_t)p[b] << (8u * (b & 3u));
    dk_u4 v;
    v.x = w[0];
    v.y = w[1];
    v.z = w[2];
    v.w = w[3];
    return v;
}

template <bool SAFE>
DK_DEV unsigned long long dk_hash(const uint8_t *k_, uint32_t n) {
    const DK_GAS uint8_t *k = (const DK_GAS uint8_t *)k_;
    unsigned long long h = 0x9E3779B97F4A7C15ull ^ n;
    for (uint32_t i = 0; i < n; i += 16) {
        const dk_u4 v = dk_load<SAFE>(k + i, n - i);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            h ^= dk_word(v, j, n - i);
            h *= 0x100000001B3ull;
        }
    }
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    return h | 1ull;
}

// a: the index's key arena (slack past its end), b: a query key (read safely)
DK_DEV bool bytes_eq(const uint8_t *a_, const uint8_t *b_, uint32_t n) {
    const DK_GAS uint8_t *a = (const DK_GAS uint8_t *)a_, *b = (const DK_GAS uint8_t *)b_;
    for (uint32_t i = 0; i < n; i += 16) {
        const dk_u4 x = dk_load<false>(a + i, n - i), y = dk_load<true>(b + i, n - i);
        uint32_t d = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) d |= dk_word(x, j, n - i) ^ dk_word(y, j, n - i);
        if (d) return false;
    }
    return true;
}

__global__ void __launch_bounds__(256) k_dk_insert(uint32_t gid0, uint32_t n, const DkRec *rec, const uint8_t *keys,
                                                   DkSlot *tab, uint32_t mask, uint32_t *err) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t gid = gid0 + j;
    const DkRec r = rec[gid];
    const uint8_t *k = keys + r.key_off;
    const unsigned long long h = dk_hash<false>(k, r.key_len);
    uint32_t i = (uint32_t)h & mask;
    for (uint32_t probes = 0; probes <= mask; ++probes, i = (i + 1) & mask) {
        // the slot of this hash: claimed by the first inserter, then every record with the
        // hash takes it, the newest id winning.  (No waiting on another inserter's id: two
        // lanes of one wave can carry the same key.  Two different keys that share all 64
        // hash bits would share the slot; a lookup verifies the key bytes, so one of them
        // then simply misses and its batch resolves on the host.)
        const unsigned long long prev = atomicCAS(&tab[i].h, 0ull, h);
        if (prev != 0ull && prev != h) continue;
        atomicMax(&tab[i].gid1, gid + 1);
        return;
    }
    atomicOr(err, 1u);  // (table full: cannot happen, it is sized at twice the records)
}

__global__ void __launch_bounds__(256) k_dk_kill(uint32_t n, const uint32_t *gids, DkRec *rec) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) rec[gids[j]].flags &= ~kDkLive;
}

// per query key (q = ticket * 256 + thread: workgroups are numbered in the order they start,
// so every predecessor a look-back waits on is running or done): its record's gather query,
// its output room in 16-byte units and its tiles; their exclusive prefix over the batch gives
// the query's output offset and first tile.  chain: two 64-bit words per workgroup (room,
// tiles), flag in the top two bits (1: this workgroup's own sum, 2: inclusive prefix), zeroed
// by the caller with ctl.
constexpr unsigned long long kChAgg = 1ull << 62, kChIncl = 2ull << 62, kChVal = (1ull << 62) - 1;
constexpr uint32_t kChSpin = 1u << 24;
__global__ void __launch_bounds__(256) k_dk_lookup(uint32_t nq, const uint8_t *qkeys, const uint64_t *qoff,
                                                   const DkSlot *tab, uint32_t mask, const DkRec *rec,
                                                   const uint8_t *keys, uint32_t mode, GatherQuery *gq,
                                                   uint32_t *out_off16, uint32_t *ctl, unsigned long long *chain,
                                                   const uint32_t *ins_err) {
    __shared__ uint32_t s_bid, s_wa[4], s_wt[4];
    __shared__ unsigned long long s_pa, s_pt;
    if (threadIdx.x == 0) s_bid = atomicAdd(&ctl[4], 1u);
    __syncthreads();
    const uint32_t bid = s_bid, q = bid * 256u + threadIdx.x, lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    bool ok = false;
    uint32_t c16 = 0, nt = 0;
    GatherQuery G{};
    if (q < nq && !*ins_err) {  // (an insert that gave up: every key goes to the host)
        const uint8_t *k = qkeys + qoff[q];
        const uint32_t n = (uint32_t)(qoff[q + 1] - qoff[q]);
        const unsigned long long h = dk_hash<true>(k, n);
        uint32_t i = (uint32_t)h & mask, g = kNone;
        for (uint32_t probes = 0; probes <= mask; ++probes, i = (i + 1) & mask) {
            const unsigned long long x = tab[i].h;
            if (x == 0ull) break;
            if (x != h) continue;
            const uint32_t g1 = tab[i].gid1;
            if (!g1) break;
            const DkRec &o = rec[g1 - 1];
            if (o.key_len == n && bytes_eq(keys + o.key_off, k, n)) {
                g = g1 - 1;
                break;
            }
        }
        if (g != kNone) {
            const DkRec r = rec[g];
            const SpanEnt *sp = mode == 0 ? r.sp : r.xsp;
            const uint32_t *t = mode == 0 ? r.t : r.xt;
            const uint32_t ns = mode == 0 ? r.n : r.xn, len = mode == 0 ? r.len : r.xlen;
            if ((r.flags & (kDkLive | kDkClean)) == (kDkLive | kDkClean) && sp) {
                const uint32_t cap = (r.doc_len + 64u + 15u) & ~15u;  // the host's out_cap
                c16 = cap / 16;
                nt = max(1u, (min(len, cap) + kGatherTile - 1) / kGatherTile);
                G = GatherQuery{sp, r.comp, 0, ns, len, cap, q, t, 0, 0};
                ok = true;
                if (len > cap) atomicAdd(&ctl[5], 1u);  // (the gather's PX_ESPACE statuses)
            }
        }
    }
    const unsigned long long m = __ballot(q < nq && !ok);
    if (m && lane == 0) atomicAdd(&ctl[0], (uint32_t)__popcll(m));
    if (bid == 0 && threadIdx.x == 0) ctl[3] = *ins_err;
    // the workgroup's inclusive scan of (room, tiles)
    uint32_t ia = c16, it = nt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t xa = __shfl_up(ia, o), xt = __shfl_up(it, o);
        if (lane >= (uint32_t)o) {
            ia += xa;
            it += xt;
        }
    }
    if (lane == 63) {
        s_wa[w] = ia;
        s_wt[w] = it;
    }
    __syncthreads();
    uint32_t pa = 0, pt = 0;
    for (uint32_t v = 0; v < w; ++v) {
        pa += s_wa[v];
        pt += s_wt[v];
    }
    if (w == 0) {  // ---- look-back over the earlier workgroups, 64 of them per step (one per lane)
        // (thread 0 alone walked back one workgroup per dependent device-scope load: the last of
        // a 10,000-key batch's 40 workgroups waited ~39 round trips -- most of the kernel)
        const unsigned long long ta = s_wa[0] + s_wa[1] + s_wa[2] + s_wa[3], tt = s_wt[0] + s_wt[1] + s_wt[2] + s_wt[3];
        unsigned long long ea = 0, et = 0;
        if (bid == 0) {
            if (lane == 0) {
                __hip_atomic_store(chain, kChIncl | ta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(chain + 1, kChIncl | tt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            if (lane == 0) {
                __hip_atomic_store(chain + 2ull * bid, kChAgg | ta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(chain + 2ull * bid + 1, kChAgg | tt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            // channel c (0: room, 1: tiles): its window's top workgroup, done flag, running sum
            int64_t top[2] = {(int64_t)bid - 1, (int64_t)bid - 1};
            bool done[2] = {false, false};
            unsigned long long sum[2] = {0ull, 0ull};
            uint32_t spins = 0;
            while (!(done[0] && done[1])) {
                bool waited = false;
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    if (done[c]) continue;  // (wave-uniform)
                    const int64_t j = top[c] - (int64_t)lane;
                    const bool valid = j >= 0;
                    const unsigned long long x =
                        valid ? __hip_atomic_load(chain + 2ull * (uint64_t)j + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                    const uint32_t f = (uint32_t)(x >> 62);
                    const unsigned long long pub = __ballot(valid && f != 0), inc = __ballot(valid && f == 2),
                                             vm = __ballot(valid);
                    // lanes [0, L]: up to the nearest inclusive prefix, or the whole window without one
                    const uint32_t L = inc ? (uint32_t)__ffsll((long long)inc) - 1u : 63u;
                    const unsigned long long need = (L == 63u ? ~0ull : ((2ull << L) - 1ull)) & vm;
                    if ((pub & need) != need) {
                        waited = true;  // (a workgroup in the range has not published yet)
                        continue;
                    }
                    unsigned long long v = ((need >> lane) & 1ull) ? (x & kChVal) : 0ull;
                    for (int o = 32; o >= 1; o >>= 1) {
                        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
                        v += (unsigned long long)lo | ((unsigned long long)hi << 32);
                    }
                    sum[c] += v;
                    if (inc) done[c] = true;
                    else top[c] -= 64;  // (every valid lane published an aggregate: the next 64)
                }
                if (waited && ++spins > kChSpin) {  // (cannot happen; the batch then goes to the host)
                    if (lane == 0) atomicAdd(&ctl[0], 1u << 30);
                    break;
                }
            }
            ea = sum[0];
            et = sum[1];
            if (lane == 0) {
                __hip_atomic_store(chain + 2ull * bid, kChIncl | (ea + ta), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(chain + 2ull * bid + 1, kChIncl | (et + tt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (lane == 0) {
            s_pa = ea;
            s_pt = et;
            if (bid == gridDim.x - 1) {
                ctl[1] = (uint32_t)(ea + ta);
                ctl[2] = (uint32_t)(et + tt);
            }
        }
    }
    __syncthreads();
    if (ok) {
        const uint64_t off = (s_pa + pa + ia - c16) * 16ull;
        G.out_off = off;
        G.tile0 = (uint32_t)(s_pt + pt + it - nt);
        gq[q] = G;
        out_off16[q] = (uint32_t)(off >> 4);  // (16-byte units: half the bytes copied down)
    }
}

// A device-resident batch's results into the caller's device arrays: byte offsets, lengths and
// statuses (px_status codes: the device codes 0..7 are the same numbers, anything else is
// PX_ECORRUPT).  Nothing is written when a key missed (ctl[0]: the host path answers that
// batch) or the output did not fit (nothing was gathered either).
__global__ void __launch_bounds__(256) k_dk_results(uint32_t n, const uint32_t *ctl, uint64_t out_cap,
                                                    const uint32_t *out_off16, const uint32_t *dl, const uint32_t *ds,
                                                    uint64_t *out_off, uint32_t *out_len, uint32_t *status) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || ctl[0] || (uint64_t)ctl[1] * 16u > out_cap) return;
    out_off[i] = (uint64_t)out_off16[i] * 16u;
    out_len[i] = dl[i];
    const uint32_t s = ctl[5] ? ds[i] : 0u;  // (statuses are only written when a query ran past its room)
    status[i] = s <= 7u ? s : 4u;
}

}  // namespace

hipError_t launch_dk_results(hipStream_t s, uint32_t n, const uint32_t *ctl, uint64_t out_cap, const uint32_t *out_off16,
                             const uint32_t *dl, const uint32_t *ds, uint64_t *out_off, uint32_t *out_len, uint32_t *status) {
    if (!n) return hipSuccess;
    k_dk_results<<<(n + 255) / 256, 256, 0, s>>>(n, ctl, out_cap, out_off16, dl, ds, out_off, out_len, status);
    return hipGetLastError();
}

hipError_t launch_dk_insert(hipStream_t s, uint32_t gid0, uint32_t n, const DkRec *rec, const uint8_t *keys, DkSlot *tab,
                            uint32_t mask, uint32_t *err) {
    if (!n) return hipSuccess;
    k_dk_insert<<<(n + 255) / 256, 256, 0, s>>>(gid0, n, rec, keys, tab, mask, err);
    return hipGetLastError();
}
hipError_t launch_dk_kill(hipStream_t s, uint32_t n, const uint32_t *gids, DkRec *rec) {
    if (!n) return hipSuccess;
    k_dk_kill<<<(n + 255) / 256, 256, 0, s>>>(n, gids, rec);
    return hipGetLastError();
}
// ctl: 32 bytes, chain: 16 bytes per 256 keys, both zeroed by the caller
hipError_t launch_dk_lookup(hipStream_t s, uint32_t nq, const uint8_t *qkeys, const uint64_t *qoff, const DkSlot *tab,
                            uint32_t mask, const DkRec *rec, const uint8_t *keys, uint32_t mode, GatherQuery *gq,
                            uint32_t *out_off16, uint32_t *ctl, unsigned long long *chain, const uint32_t *ins_err) {
    if (!nq) return hipSuccess;
    k_dk_lookup<<<(nq + 255) / 256, 256, 0, s>>>(nq, qkeys, qoff, tab, mask, rec, keys, mode, gq, out_off16, ctl, chain,
                                                 ins_err);
    return hipGetLastError();
}

}  // namespace px
