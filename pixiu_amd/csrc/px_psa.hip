// px_psa.hip — the GST walk of setitem restated as suffix-array work.
//
// The reference inserts every doc byte into an online generalized suffix tree
// (SuffixTree.cpp:144-289) and hands the stream encoder one message per byte
// (SuffixTree.cpp:136-142, 183, 186).  Its active point after byte i of doc `cur` is the
// longest suffix of cur[0..i] that occurs earlier in the live chunk, and the edge label
// it reports is the first leaf created under that point, i.e. the earliest occurrence
// (leaves are created in (doc, start) order, splits keep the upper label:
// SuffixTree.cpp:154-157, 196-222).  With lpf(j) = the longest prefix of T[j..doc end)
// occurring at an earlier start of the shard text T (the Longest Previous Factor):
//   * byte i is COMPRESS iff lpf(i) >= 1, except at i = j-1 + lpf(j-1) for every j
//     whose lpf(j) >= lpf(j-1) (there the active point restarts: a PASS);
//   * the COMPRESS run started by j has lpf(j) - lpf(j-1) bytes and ends at
//     b = j + lpf(j) - 1 with message (doc, pos) = the earliest occurrence E of
//     T[j .. j+lpf(j)): pos = E + lpf(j) - 1 (and one byte shorter at b-1 when T[b] is a
//     251 that the encoder's pair rule can cut, PiXiuStr.cpp:33-54).
// Only runs of >= 7 bytes become reference tokens (PiXiuStr.cpp:56-82), so only those
// ends need E.  The stream is the textbook Ukkonen walk's; the reference differs from it
// only when its stale (act_chunk_idx, act_direct) pair is read (SuffixTree.cpp:171,184 vs
// the canonisation at 232-249), which needs a PASS step whose split loop stops inside an
// edge -- possible only when the restarted factor's earliest occurrence ends at a doc
// end.  Such shards are flagged and walked by k_gst_encode instead.
//
// Pipeline over all PSA shards of a batch (one global position space, shard-major):
//   k_psa_gather   docs -> global text G + doc id per position
//   k_psa_key0     5-symbol keys (shard in the top bits) -> radix sort (rocPRIM)
//   prefix doubling: keys (group, rank[p+h]) of unsorted suffixes only, stable radix
//                  sort, group heads by max-scans, ranks and SA written back
//   k_psa_minlvl / k_psa_ansv   nearest smaller position left/right in SA order
//                  (a 64-ary min tree; one wave per 64 ranks, ballot descents)
//   k_psa_lce      lcp with those two neighbours, Kasai-style in text order
//                  (lcp(p) >= lcp(p-1) - 1 for both neighbours)
//   k_psa_msg0 / k_psa_runs   messages, earliest occurrences (neighbour chains), the
//                  stale-pair check; k_psa_place   chunk / slot / status per record
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "px_common.h"

namespace px {

namespace {

constexpr uint32_t kNoPos = 0xffffffffu;
constexpr uint32_t kPass = 0xffffffffu;
#define PSA_DEV __device__ __forceinline__
#define PX_GAS __attribute__((address_space(1)))

PSA_DEV uint32_t lane_id() { return threadIdx.x & 63u; }

// ---------------------------------------------------------------- text
// G = the text, pdoc = doc id and dist = bytes to the doc's end, per position
__global__ void __launch_bounds__(256) k_psa_gather(uint32_t ndocs, const PsaDoc *docs, uint8_t *G, uint32_t *pdoc,
                                                    uint16_t *dist) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t g = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); g < ndocs; g += waves) {
        const PsaDoc d = docs[g];
        const PX_GAS uint8_t *src = (const PX_GAS uint8_t *)d.src;
        for (uint32_t o = lane; o < d.len; o += 64) {
            G[d.start + o] = src[o];
            pdoc[d.start + o] = g;
            dist[d.start + o] = (uint16_t)(d.len - o);  // 1..65,535
        }
    }
}

// initial keys: shard (top bits) | `syms` symbols of 9 bits (byte + 1; 0 past the doc end):
// as many symbols as the shard count leaves room for (5 to 6)
__global__ void __launch_bounds__(256) k_psa_key0(uint32_t N, const uint8_t *G, const uint32_t *pdoc,
                                                  const PsaDoc *docs, const uint16_t *dist, uint32_t syms,
                                                  uint64_t *keys, uint32_t *vals) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    const uint32_t left = dist[p];
    uint64_t k = (uint64_t)docs[pdoc[p]].shard << (9 * syms);
    for (uint32_t s = 0; s < syms; ++s) {
        const uint64_t sym = s < left ? (uint64_t)G[p + s] + 1 : 0;
        k |= sym << (9 * (syms - 1 - s));
    }
    keys[p] = k;
    vals[p] = p;
}

// group heads of the first sort: a new group at a key change, and every suffix shorter
// than 5 symbols (its key holds its whole string: equal ones are equal strings, kept
// in position order by the stable sort and resolved as they are)
__global__ void __launch_bounds__(256) k_psa_head0(uint32_t N, const uint64_t *keys, const uint32_t *sa,
                                                   const uint16_t *dist, uint32_t syms, uint32_t *hflag) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    const uint32_t p = sa[r];
    const bool complete = dist[p] < syms;
    hflag[r] = (r == 0 || keys[r] != keys[r - 1] || complete) ? r : 0u;
}

// rank = group head index; active = not a singleton group
__global__ void __launch_bounds__(256) k_psa_rank0(uint32_t N, const uint32_t *sa, const uint32_t *head,
                                                   uint32_t *rank, uint8_t *active) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    rank[sa[r]] = head[r];
    const bool h = head[r] == r;
    const bool hn = r + 1 == N || head[r + 1] == r + 1;
    active[r] = (h && hn) ? 0 : 1;
}

// doubling step h: key (group, rank of the suffix h further, 0 past the doc end)
__global__ void __launch_bounds__(256) k_psa_key2(uint32_t m, const uint32_t *act, const uint32_t *rank,
                                                  const uint16_t *dist, uint32_t h, uint64_t *keys, uint32_t *vals) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    const uint32_t p = act[t];
    const uint64_t hi = rank[p];
    const uint64_t lo = h < dist[p] ? (uint64_t)rank[p + h] + 1 : 0;
    keys[t] = hi << 32 | lo;
    vals[t] = p;
}

__global__ void __launch_bounds__(256) k_psa_head2(uint32_t m, const uint64_t *keys, uint32_t *gflag, uint32_t *sflag) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    const uint64_t k = keys[t];
    const bool first = t == 0;
    gflag[t] = (first || (k >> 32) != (keys[t - 1] >> 32)) ? t : 0u;
    // a suffix whose string ended (lo == 0) is complete: its own group
    sflag[t] = (first || k != keys[t - 1] || (uint32_t)k == 0) ? t : 0u;
}

__global__ void __launch_bounds__(256) k_psa_rank2(uint32_t m, const uint64_t *keys, const uint32_t *pos,
                                                   const uint32_t *gfirst, const uint32_t *sfirst, uint32_t *sa,
                                                   uint32_t *rank, uint8_t *active) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    const uint64_t k = keys[t];
    const uint32_t g = (uint32_t)(k >> 32);
    const uint32_t p = pos[t];
    sa[g + (t - gfirst[t])] = p;
    rank[p] = g + (sfirst[t] - gfirst[t]);
    const bool h = sfirst[t] == t;
    const bool hn = t + 1 == m || keys[t + 1] != k || (uint32_t)keys[t + 1] == 0;
    active[t] = (h && hn) ? 0 : 1;
}

// ---------------------------------------------------------------- segmented doubling sort
// A doubling step's keys arrive in suffix-array order, so each group (equal high word) is
// a contiguous range and only needs sorting by the low word inside it.  From the third
// step on almost every group is small (config 3: every group <= 113 suffixes from h = 24
// on, 90 % of suffixes in groups <= 1,024 at h = 12), so groups are sorted where they lie:
// <= 64 by one wave (bitonic over lanes), <= kSegBlock by one workgroup (bitonic in LDS),
// and only the rest go through the global radix sort.  Ties (equal low words: identical
// complete strings) keep their input order, as the stable radix sort keeps them.
constexpr uint32_t kSegBlock = 1024;

__global__ void __launch_bounds__(256) k_seg_flag(uint32_t m, const uint64_t *keys, uint8_t *fl) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    fl[t] = (t == 0 || (keys[t] >> 32) != (keys[t - 1] >> 32)) ? 1 : 0;
}

// group sizes -> size classes: c < 6: size <= 2^(c+1) (sorted 64 / 2^(c+1) groups per
// wave), 6: <= kSegBlock (one workgroup), 7: larger (radix).  The class lists are one
// array partitioned class-major: per-block class counts, one exclusive scan over them
// (class-major), then every block writes its groups at its offsets.
constexpr int kSegClasses = 8;
PSA_DEV uint32_t seg_class_of(uint32_t g, uint32_t ng, const uint32_t *gs, uint32_t m) {
    const uint32_t sz = (g + 1 < ng ? gs[g + 1] : m) - gs[g];
    uint32_t c = sz <= kSegBlock ? 6 : 7;
    for (int k = 5; k >= 0; --k)
        if (sz <= (2u << k)) c = (uint32_t)k;
    return c;
}
__global__ void __launch_bounds__(256) k_seg_hist(uint32_t ng, const uint32_t *gs, uint32_t m, uint32_t nb,
                                                  uint32_t *hist) {
    __shared__ uint32_t h[kSegClasses];
    if (threadIdx.x < kSegClasses) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < ng) atomicAdd(&h[seg_class_of(g, ng, gs, m)], 1u);
    __syncthreads();
    if (threadIdx.x < kSegClasses) hist[threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}
__global__ void __launch_bounds__(256) k_seg_part(uint32_t ng, const uint32_t *gs, uint32_t m, uint32_t nb,
                                                  const uint32_t *offs, uint32_t *lists) {
    __shared__ uint32_t h[kSegClasses];
    if (threadIdx.x < kSegClasses) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < ng) {
        const uint32_t c = seg_class_of(g, ng, gs, m);
        lists[offs[c * nb + blockIdx.x] + atomicAdd(&h[c], 1u)] = g;  // order inside a class is free
    }
}
// class start offsets -> out[0..8] (out[8] = ng)
__global__ void k_seg_bounds(uint32_t nb, const uint32_t *offs, uint32_t ng, uint32_t *out) {
    const uint32_t c = threadIdx.x;
    if (c < kSegClasses) out[c] = offs[c * nb];
    if (c == kSegClasses) out[c] = ng;
}

PSA_DEV void cas_shfl(uint64_t &k, uint32_t &v, uint32_t lane, uint32_t j, bool up) {
    const uint64_t ok = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(k >> 32), (int)j) << 32) |
                        (uint32_t)__shfl_xor((int)(uint32_t)k, (int)j);
    const uint32_t ov = (uint32_t)__shfl_xor((int)v, (int)j);
    const bool lower = (lane & j) == 0;
    const bool take = up == lower ? ok < k : ok > k;
    if (take) {
        k = ok;
        v = ov;
    }
}

// groups of <= S suffixes, 64 / S per wave: bitonic over S-lane segments, sort key
// (low word << 6 | input index)
template <uint32_t S>
__global__ void __launch_bounds__(256) k_seg_sortS(uint32_t n, const uint32_t *list, const uint32_t *gs, uint32_t ng,
                                                   uint32_t m, const uint64_t *keys, const uint32_t *vals,
                                                   uint64_t *keys_out, uint32_t *vals_out) {
    // grid-stride: a dispatch holds fewer than 2^32 work-items, and there can be ~10^8 groups
    constexpr uint32_t G = 64 / S;
    const uint32_t lane = lane_id(), i = lane & (S - 1);
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); w * G < n; w += waves) {
        const uint32_t slot = w * G + lane / S;
        uint32_t a = 0, sz = 0;
        if (slot < n) {
            const uint32_t g = list[slot];
            a = gs[g];
            sz = (g + 1 < ng ? gs[g + 1] : m) - a;
        }
        uint64_t k = ~0ull, hi = 0;
        uint32_t v = 0;
        if (i < sz) {
            const uint64_t key = keys[a + i];
            hi = key >> 32;
            k = (key & 0xffffffffull) << 6 | i;
            v = vals[a + i];
        }
        for (uint32_t kk = 2; kk <= S; kk <<= 1)
            for (uint32_t j = kk >> 1; j > 0; j >>= 1) cas_shfl(k, v, lane, j, (i & kk) == 0);
        if (i < sz) {
            keys_out[a + i] = hi << 32 | (k >> 6);
            vals_out[a + i] = v;
        }
    }
}

// one workgroup per group of 65..kSegBlock: bitonic sort in LDS
__global__ void __launch_bounds__(256) k_seg_sortblk(const uint32_t *list, const uint32_t *gs, uint32_t ng, uint32_t m,
                                                     const uint64_t *keys, const uint32_t *vals, uint64_t *keys_out,
                                                     uint32_t *vals_out) {
    __shared__ uint64_t sk[kSegBlock];
    __shared__ uint32_t sv[kSegBlock];
    const uint32_t g = list[blockIdx.x];
    const uint32_t a = gs[g], sz = (g + 1 < ng ? gs[g + 1] : m) - a;
    uint32_t P = 128;
    while (P < sz) P <<= 1;
    const uint64_t hi = keys[a] >> 32;
    for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
        if (i < sz) {
            sk[i] = (keys[a + i] & 0xffffffffull) << 10 | i;
            sv[i] = vals[a + i];
        } else {
            sk[i] = ~0ull;
            sv[i] = 0;
        }
    }
    __syncthreads();
    for (uint32_t kk = 2; kk <= P; kk <<= 1)
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const bool up = (i & kk) == 0;
                    const uint64_t x = sk[i], y = sk[l];
                    if (up ? x > y : x < y) {
                        sk[i] = y;
                        sk[l] = x;
                        const uint32_t t = sv[i];
                        sv[i] = sv[l];
                        sv[l] = t;
                    }
                }
            }
            __syncthreads();
        }
    for (uint32_t i = threadIdx.x; i < sz; i += blockDim.x) {
        keys_out[a + i] = hi << 32 | (sk[i] >> 10);
        vals_out[a + i] = sv[i];
    }
}

// big groups: mark their elements, then gather / radix sort / scatter back
__global__ void __launch_bounds__(256) k_seg_mark(const uint32_t *list, const uint32_t *gs, uint32_t ng, uint32_t m,
                                                  uint8_t *fl) {
    const uint32_t g = list[blockIdx.x];
    const uint32_t a = gs[g], sz = (g + 1 < ng ? gs[g + 1] : m) - a;
    for (uint32_t i = threadIdx.x; i < sz; i += blockDim.x) fl[a + i] = 1;
}
__global__ void __launch_bounds__(256) k_seg_gather(uint32_t n, const uint32_t *idx, const uint64_t *keys,
                                                    const uint32_t *vals, uint64_t *ck, uint32_t *cv) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    ck[i] = keys[idx[i]];
    cv[i] = vals[idx[i]];
}
__global__ void __launch_bounds__(256) k_seg_scatter(uint32_t n, const uint32_t *idx, const uint64_t *ck,
                                                     const uint32_t *cv, uint64_t *keys_out, uint32_t *vals_out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys_out[idx[i]] = ck[i];
    vals_out[idx[i]] = cv[i];
}

// ---------------------------------------------------------------- stream compaction
// out = values[i] (or i itself when values is null) for every i < n with flags[i] != 0, in
// order.  Three passes: per-tile counts, a scan over the tiles, per-tile writes.  A
// tile is 4,096 elements (16 per thread, read as one 16-byte flag vector).
constexpr uint32_t kCmpTile = 4096;
PSA_DEV uint32_t nflags16(const uint8_t *f, uint32_t i, uint32_t n, uint32_t &bits) {
    bits = 0;
    if (i + 16 <= n) {
        const uint4 v = *(const uint4 *)(f + i);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int q = 0; q < 4; ++q)
            for (int b = 0; b < 4; ++b)
                if ((w[q] >> (8 * b)) & 0xffu) bits |= 1u << (4 * q + b);
    } else {
        for (uint32_t k = 0; k < 16 && i + k < n; ++k)
            if (f[i + k]) bits |= 1u << k;
    }
    return (uint32_t)__popc(bits);
}
__global__ void __launch_bounds__(256) k_cmp_count(uint32_t n, const uint8_t *flags, uint32_t *tile_cnt) {
    __shared__ uint32_t red[4];
    const uint32_t i = blockIdx.x * kCmpTile + threadIdx.x * 16;
    uint32_t bits;
    uint32_t c = i < n ? nflags16(flags, i, n, bits) : 0;
    for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ void __launch_bounds__(256) k_cmp_write(uint32_t n, const uint8_t *flags, const uint32_t *values,
                                                   const uint32_t *tile_off, uint32_t *out) {
    __shared__ uint32_t wsum[4];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * kCmpTile + threadIdx.x * 16;
    uint32_t bits = 0;
    const uint32_t c = i < n ? nflags16(flags, i, n, bits) : 0;
    // exclusive prefix of c over the block
    uint32_t x = c;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if ((int)lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t base = tile_off[blockIdx.x] + x - c;
    for (uint32_t k = 0; k < wv; ++k) base += wsum[k];
    if (!bits) return;
    if (values && i + 16 <= n) {
        uint32_t v[16];
        for (int q = 0; q < 4; ++q) *(uint4 *)(v + 4 * q) = *(const uint4 *)(values + i + 4 * q);
        for (uint32_t k = 0; k < 16; ++k)
            if (bits >> k & 1u) out[base++] = v[k];
    } else {
        for (uint32_t k = 0; k < 16; ++k)
            if (bits >> k & 1u) out[base++] = values ? values[i + k] : i + k;
    }
}

__global__ void k_cmp_total(uint32_t nt, const uint32_t *tile_cnt, const uint32_t *tile_off, uint32_t *total) {
    *total = nt ? tile_off[nt - 1] + tile_cnt[nt - 1] : 0;
}

// debug (PX_PSA_SEGCHECK=1): compare the segmented sort with the radix sort
__global__ void k_seg_cmp(uint32_t m, const uint64_t *k1, const uint32_t *v1, const uint64_t *k2, const uint32_t *v2,
                          uint32_t *out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    if (k1[t] != k2[t] || v1[t] != v2[t]) {
        const uint32_t c = atomicAdd(&out[0], 1u);
        if (c == 0) {
            out[1] = t;
        }
    }
}

// ---------------------------------------------------------------- nearest smaller positions
// 64-ary min tree over the suffix array's values (text positions)
__global__ void __launch_bounds__(256) k_psa_minlvl(uint32_t n_in, const uint32_t *in, uint32_t n_out, uint32_t *out) {
    const uint32_t lane = lane_id();
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w >= n_out) return;
    const uint32_t i = w * 64 + lane;
    uint32_t v = i < n_in ? in[i] : kNoPos;
    for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
    if (lane == 0) out[w] = v;
}

struct MinTree {
    const uint32_t *lvl[8];
    uint32_t n[8];
    uint32_t levels;  // lvl[0] = the suffix array
};

// nearest index left (dir 0) / right (dir 1) of element i whose value is < v, or kNoPos
// (wave-cooperative: every lane calls it with the same i and v)
PSA_DEV uint32_t tree_find(const MinTree &t, uint32_t i, uint32_t v, int dir) {
    const uint32_t lane = lane_id();
    uint32_t x = i;  // node index at level L
    for (uint32_t L = 0; L < t.levels; ++L) {
        const uint32_t base = x & ~63u, at = x & 63u;
        const uint32_t j = base + lane;
        const uint32_t s = j < t.n[L] ? t.lvl[L][j] : kNoPos;
        const bool side = dir == 0 ? lane < at : lane > at;
        const uint64_t mm = __ballot(side && s < v);
        if (mm) {
            uint32_t y = base + (dir == 0 ? 63u - (uint32_t)__clzll((long long)mm) : (uint32_t)__ffsll((long long)mm) - 1u);
            for (uint32_t D = L; D-- > 0;) {  // descend to the element
                const uint32_t c = y * 64 + lane;
                const uint32_t cv = c < t.n[D] ? t.lvl[D][c] : kNoPos;
                const uint64_t cm = __ballot(cv < v);
                y = y * 64 + (dir == 0 ? 63u - (uint32_t)__clzll((long long)cm) : (uint32_t)__ffsll((long long)cm) - 1u);
            }
            return y;
        }
        x >>= 6;
    }
    return kNoPos;
}

// psv / nsv: for the suffix at rank r, the nearest rank to its left / right (inside its
// shard's range) whose position is smaller; written per position
// the shard whose range holds suffix-array index r (shards are contiguous and in order in
// both position and rank space)
PSA_DEV uint32_t shard_of_rank(const PsaShard *shards, uint32_t nshards, uint32_t r) {
    uint32_t a = 0, b = nshards;  // shards[a].base <= r < shards[b].base
    while (b - a > 1) {
        const uint32_t c = (a + b) >> 1;
        if (shards[c].base <= r) a = c;
        else b = c;
    }
    return a;
}

__global__ void __launch_bounds__(256) k_psa_ansv(uint32_t N, MinTree t, const PsaShard *shards, uint32_t nshards,
                                                  uint2 *links) {
    const uint32_t lane = lane_id();
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (w * 64 >= N) return;
    const uint32_t *sa = t.lvl[0];
    const uint32_t r = w * 64 + lane;
    const bool live = r < N;
    const uint32_t v = live ? sa[r] : kNoPos;
    // this block of 64 ranks lies in one shard unless it straddles a boundary
    const uint32_t r0 = w * 64, r1 = min(N, r0 + 64) - 1;
    const uint32_t s0 = shard_of_rank(shards, nshards, __builtin_amdgcn_readfirstlane(r0));
    const PsaShard sh0 = shards[s0];
    uint32_t lo = sh0.base, hi = sh0.base + sh0.len;
    if (r1 >= hi && live && r >= hi) {
        const PsaShard sh = shards[shard_of_rank(shards, nshards, r)];
        lo = sh.base;
        hi = sh.base + sh.len;
    }
    // inside the 64-rank block: binary lifting over window minima.  ml[k] = min of the
    // 2^k lanes ending at this lane, mr[k] = of the 2^k lanes starting at it
    uint32_t ml[6], mr[6];
    ml[0] = mr[0] = v;
    for (int k = 1; k < 6; ++k) {
        const uint32_t w = 1u << (k - 1);
        const uint32_t a = (uint32_t)__shfl((int)ml[k - 1], (int)((lane - w) & 63u));
        const uint32_t b = (uint32_t)__shfl((int)mr[k - 1], (int)((lane + w) & 63u));
        ml[k] = lane >= w ? min(ml[k - 1], a) : ml[k - 1];
        mr[k] = lane + w < 64 ? min(mr[k - 1], b) : mr[k - 1];
    }
    // nearest smaller to the left: extend (pl, lane) while its minimum stays >= v
    int pl = (int)lane - 1, pr = (int)lane + 1;
    for (int k = 5; k >= 0; --k) {
        const int w = 1 << k;
        const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(max(pl, 0) << 2, (int)ml[k]);
        if (pl - w + 1 >= 0 && a >= v) pl -= w;
        const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(min(pr, 63) << 2, (int)mr[k]);
        if (pr + w - 1 <= 63 && b >= v) pr += w;
    }
    uint32_t ps = pl >= 0 ? r - (lane - (uint32_t)pl) : kNoPos;
    uint32_t ns = pr <= 63 ? r + ((uint32_t)pr - lane) : kNoPos;
    if (ns != kNoPos && ns >= N) ns = kNoPos;
    // the rest through the min tree, one element at a time (few per block: the block's
    // prefix / suffix minima)
    uint64_t need = __ballot(live && (ps == kNoPos || ns == kNoPos));
    while (need) {
        const uint32_t l = (uint32_t)__ffsll((long long)need) - 1u;
        need &= need - 1;
        const uint32_t ri = w * 64 + l;
        const uint32_t vi = (uint32_t)__shfl((int)v, (int)l);
        const uint32_t pi = (uint32_t)__shfl((int)ps, (int)l);
        const uint32_t ni = (uint32_t)__shfl((int)ns, (int)l);
        const uint32_t fp = pi == kNoPos ? tree_find(t, ri, vi, 0) : pi;
        const uint32_t fn = ni == kNoPos ? tree_find(t, ri, vi, 1) : ni;
        if (lane == l) {
            ps = fp;
            ns = fn;
        }
    }
    if (live)  // in rank order (coalesced); k_psa_links_text moves them to text order
        links[r] = make_uint2((ps != kNoPos && ps >= lo) ? sa[ps] : kNoPos, (ns != kNoPos && ns < hi) ? sa[ns] : kNoPos);
}

// the links in text order: one scattered 8-byte read per position instead of two
// scattered 4-byte writes in k_psa_ansv (rank = the inverse suffix array)
__global__ void __launch_bounds__(256) k_psa_links_text(uint32_t N, const uint32_t *rank, const uint2 *links,
                                                        uint32_t *psvp, uint32_t *nsvp) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    const uint2 l = links[rank[p]];
    psvp[p] = l.x;
    nsvp[p] = l.y;
}

// ---------------------------------------------------------------- lcp with those neighbours
// text positions per thread (Kasai-style amortisation): 256, or fewer (a multiple of 8)
// when that leaves fewer than 2^18 threads -- a one-chunk window of the single instance
constexpr uint32_t kLceSpan = 256;
inline uint32_t lce_span(uint64_t n) {
    uint64_t sp = kLceSpan;
    while (sp > 16 && n / sp < (1u << 18)) sp /= 2;
    return (uint32_t)sp;
}

// 8 text bytes from any offset: two aligned 8-byte loads and a funnel shift
PSA_DEV uint64_t ld8(const uint64_t *G8, uint32_t off) {
    const uint32_t w = off >> 3, sh = (off & 7u) * 8u;
    const uint64_t a = G8[w];
    if (!sh) return a;
    const uint64_t b = G8[w + 1];
    return (a >> sh) | (b << (64u - sh));
}

PSA_DEV uint32_t lce(const uint64_t *G8, uint32_t p, uint32_t q, uint32_t k, uint32_t lim) {
    // bytes equal from offset k on, up to lim (both suffixes stay inside their docs)
    while (k < lim) {
        const uint64_t x = ld8(G8, p + k) ^ ld8(G8, q + k);
        if (x) return min(lim, k + (uint32_t)(__builtin_ctzll(x) >> 3));
        k += 8;
    }
    return lim;
}

// One thread per `span` consecutive positions.  The per-position arrays are read and
// written 8 positions at a time with 16-byte accesses: a wave's 64 threads sit 256
// positions apart, so per-position 2- and 4-byte accesses would each touch a different
// cache line (and 64 threads x 5 arrays of such lines do not stay cached between the
// thread's consecutive positions).
__global__ void __launch_bounds__(256) k_psa_lce(uint32_t N, const uint64_t *G8, const uint16_t *dist,
                                                 const uint32_t *psvp, const uint32_t *nsvp, uint16_t *lcp_p,
                                                 uint16_t *lcp_n, uint32_t span) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t p0 = t * span;
    if (p0 >= N) return;
    const uint32_t p1 = min(N, p0 + span);
    uint32_t kp = 0, kn = 0, qprev = kNoPos - 1, sprev = kNoPos - 1;
    for (uint32_t b = p0; b < p1; b += 8) {
        const uint32_t nb = min(8u, p1 - b);
        uint16_t dv[8], op[8], on[8];
        uint32_t qv[8], sv[8];
        if (nb == 8) {  // b is a multiple of 8: aligned vector loads
            *(uint4 *)dv = *(const uint4 *)(dist + b);
            *(uint4 *)qv = *(const uint4 *)(psvp + b);
            *(uint4 *)(qv + 4) = *(const uint4 *)(psvp + b + 4);
            *(uint4 *)sv = *(const uint4 *)(nsvp + b);
            *(uint4 *)(sv + 4) = *(const uint4 *)(nsvp + b + 4);
        } else {
            for (uint32_t i = 0; i < nb; ++i) {
                dv[i] = dist[b + i];
                qv[i] = psvp[b + i];
                sv[i] = nsvp[b + i];
            }
        }
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            if (i >= nb) break;
            const uint32_t p = b + i, dp = dv[i], q = qv[i], sn = sv[i];
            // the shifted pair: lcp(p-1, q') = L >= 2 gives lcp(p, q'+1) = L - 1 exactly
            // (same mismatch, or the same doc end, one byte on; both stay in their docs),
            // so a neighbour that continues the previous one needs no text at all
            const bool shp = q != kNoPos && q == qprev + 1 && kp >= 2;
            const bool shn = sn != kNoPos && sn == sprev + 1 && kn >= 2;
            kp = kp ? kp - 1 : 0;
            kn = kn ? kn - 1 : 0;
            if (q == kNoPos) {
                kp = 0;
            } else if (!shp) {
                const uint32_t lim = min(dp, (uint32_t)dist[q]);
                kp = lce(G8, p, q, min(kp, lim), lim);
            }
            if (sn == kNoPos) {
                kn = 0;
            } else if (!shn) {
                const uint32_t lim = min(dp, (uint32_t)dist[sn]);
                kn = lce(G8, p, sn, min(kn, lim), lim);
            }
            qprev = q;
            sprev = sn;
            op[i] = (uint16_t)kp;
            on[i] = (uint16_t)kn;
        }
        if (nb == 8) {
            *(uint4 *)(lcp_p + b) = *(const uint4 *)op;
            *(uint4 *)(lcp_n + b) = *(const uint4 *)on;
        } else {
            for (uint32_t i = 0; i < nb; ++i) {
                lcp_p[b + i] = op[i];
                lcp_n[b + i] = on[i];
            }
        }
    }
}

// ---------------------------------------------------------------- messages
PSA_DEV uint32_t lpf_at(const uint16_t *lp, const uint16_t *ln, uint32_t p) { return max((uint32_t)lp[p], (uint32_t)ln[p]); }

// earliest occurrence of T[j .. j+l): climb the nearest-smaller-position links while the
// neighbour still shares l symbols (positions strictly decrease)
PSA_DEV uint32_t earliest(const uint32_t *psvp, const uint32_t *nsvp, const uint16_t *lp, const uint16_t *ln, uint32_t j,
                          uint32_t l) {
    uint32_t p = j;
    for (;;) {
        if (lp[p] >= l) p = psvp[p];
        else if (ln[p] >= l) p = nsvp[p];
        else return p;
    }
}

PSA_DEV uint32_t msg_of(const PsaDoc *docs, const uint32_t *pdoc, uint32_t e, uint32_t l) {
    const PsaDoc &d = docs[pdoc[e]];
    return d.slot << 16 | (e - d.start + l - 1);
}

// every byte of a new doc: COMPRESS (placeholder 0) when lpf >= 1, else PASS
__global__ void __launch_bounds__(256) k_psa_msg0(uint32_t N, const uint32_t *pdoc, const PsaDoc *docs,
                                                  const uint16_t *lp, const uint16_t *ln) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    const PsaDoc &d = docs[pdoc[p]];
    if (!d.msg) return;
    d.msg[p - d.start] = lpf_at(lp, ln, p) >= 1 ? 0u : kPass;
}

__global__ void __launch_bounds__(256) k_psa_runs(uint32_t N, const uint8_t *G, const uint32_t *pdoc, const PsaDoc *docs,
                                                  const uint16_t *dist, const uint32_t *psvp, const uint32_t *nsvp,
                                                  const uint16_t *lp, const uint16_t *ln, uint32_t *shard_flag) {
    const uint32_t J = blockIdx.x * blockDim.x + threadIdx.x;
    if (J >= N) return;
    const uint32_t g = pdoc[J];
    const PsaDoc &d = docs[g];
    const uint32_t end = d.start + d.len;
    const uint32_t lJ = lpf_at(lp, ln, J);
    const uint32_t lq = J > d.start ? lpf_at(lp, ln, J - 1) : 0;
    const bool restart = J > d.start && lJ >= lq;  // a non-empty active-point range starts at J
    if (d.msg) {
        if (restart && J - 1 + lq < end) d.msg[J - 1 + lq - d.start] = kPass;
        if (lJ >= lq + 7) {  // a COMPRESS run of >= 7 bytes: a reference token can end here
            const uint32_t b = J + lJ - 1;
            d.msg[b - d.start] = msg_of(docs, pdoc, earliest(psvp, nsvp, lp, ln, J, lJ), lJ);
            if (G[b] == 251) d.msg[b - 1 - d.start] = msg_of(docs, pdoc, earliest(psvp, nsvp, lp, ln, J, lJ - 1), lJ - 1);
        }
        // stale-pair check (see the file comment): the restart at J-1+lq leaves the split
        // loop inside an edge only if T[J-1 .. J-1+lq)'s earliest occurrence ends its doc
        if (restart && lq >= 2) {
            const uint32_t fe = J - 1 + lq;
            if (G[fe - 2] == 251 && (G[fe - 1] == 0 || G[fe - 1] == 2)) {
                const uint32_t e = earliest(psvp, nsvp, lp, ln, J - 1, lq);
                if (lq == dist[e]) shard_flag[d.shard] = 1;
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_psa_place(uint32_t ndocs, const PsaDoc *docs, const PsaShard *shards,
                                                   uint32_t *rec_chunk, uint32_t *rec_idx, uint32_t *rec_status) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= ndocs) return;
    const PsaDoc d = docs[g];
    if (!d.msg) return;
    rec_chunk[d.rec] = shards[d.shard].chunk;
    rec_idx[d.rec] = d.slot;
    rec_status[d.rec] = kOk;
}

// ---------------------------------------------------------------- MemPool emulation
// The walk charges MemPool blocks per leaf it creates (MemPool.cpp:7-37; SuffixTree.cpp:
// 148-227): a leaf under the root or under an existing node [5, 3] (STNode 40 B, child-map
// entry 24 B), a leaf that splits an edge [5, 5, 3, 3] (leaf, inner node, two entries).
// Leaf j of a doc ending at e exists iff j + lpf(j) < e; leaves are created in position
// order.  With sigma = T[j .. j+lpf(j)), E its earliest occurrence and a = T[E + |sigma|]:
// sigma is already a node iff an earlier leaf had the same sigma or E's doc ends right after
// sigma (E's leaf node).  The leaves with a given sigma are the first occurrences of
// sigma.c (c != a), so the split happens at the smallest of them: the minimum of sigma's
// suffix-array interval outside sigma.a's.  That is the minimum of one side of sigma.a,
// and a side minimum has its nearest smaller position on one side outside sigma (or among
// the terminated copies of sigma, which sort first and are implicit doc ends, not leaves)
// and on the other inside sigma.a: at most two candidates per sigma, the smaller splits.
// (tools/proto/pool_proto.cpp is the CPU prototype, checked doc by doc against the walk.)
// code: 0 no leaf, 1 leaf [5, 3], 2 split candidate, 3 split leaf [5, 5, 3, 3]
// the links of one position packed for the candidates' climbs: one 16-byte load per step
struct alignas(16) LinkRec {
    uint32_t psv, nsv;
    uint16_t lp, ln, dist, pad;
};
__global__ void __launch_bounds__(256) k_pool_pack(uint32_t N, const uint32_t *psvp, const uint32_t *nsvp,
                                                   const uint16_t *lp, const uint16_t *ln, const uint16_t *dist,
                                                   LinkRec *rec) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    rec[p] = LinkRec{psvp[p], nsvp[p], lp[p], ln[p], dist[p], 0};
}
__global__ void __launch_bounds__(256) k_pool_leaf(uint32_t N, const uint8_t *G, const uint32_t *pdoc, const PsaDoc *docs,
                                                   const PsaShard *shards, const LinkRec *R, uint8_t *code, uint32_t *E,
                                                   uint32_t *ncand) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t c = 0;
    if (p < N) {
        const PsaDoc &d = docs[pdoc[p]];
        if (shards[d.shard].pools) {
            const LinkRec me = R[p];
            const uint32_t l = max(me.lp, me.ln);
            if (p + l < d.start + d.len) {
                c = 1;
                if (l) {
                    uint32_t q = kNoPos;
                    if (me.ln < l) q = me.psv;
                    else if (me.lp < l || R[me.psv].dist == l) q = me.nsv;
                    if (q != kNoPos) {
                        // climb to E = the earliest occurrence of T[q .. q+l), keeping q's record
                        LinkRec rq = R[q], r = rq;
                        uint32_t e = q;
                        for (;;) {
                            if (r.lp >= l) e = r.psv;
                            else if (r.ln >= l) e = r.nsv;
                            else break;
                            r = R[e];
                        }
                        if (r.dist > l && rq.dist > l && G[q + l] == G[e + l]) {
                            c = 2;
                            E[p] = e;
                        }
                    }
                }
            }
        }
        code[p] = (uint8_t)c;
    }
    const uint64_t m = __ballot(c == 2);
    if (lane_id() == 0 && m) atomicAdd(ncand, (uint32_t)__popcll(m));
}

struct PoolSlot {
    unsigned long long key;  // (E << 16 | l), ~0: empty
    uint32_t min;            // smallest candidate position
    uint32_t pad;
};
PSA_DEV uint32_t pool_hash(uint64_t k, uint32_t mask) {
    k *= 0x9E3779B97F4A7C15ull;
    return (uint32_t)(k >> 32) & mask;
}
__global__ void __launch_bounds__(256) k_pool_insert(uint32_t N, const uint8_t *code, const uint32_t *E, const uint16_t *lp,
                                                     const uint16_t *ln, PoolSlot *tab, uint32_t mask) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N || code[p] != 2) return;
    const unsigned long long key = (unsigned long long)E[p] << 16 | max(lp[p], ln[p]);
    for (uint32_t h = pool_hash(key, mask);; h = (h + 1) & mask) {
        const unsigned long long old = atomicCAS(&tab[h].key, ~0ull, key);
        if (old == ~0ull || old == key) {
            atomicMin(&tab[h].min, p);
            return;
        }
    }
}
// split decision and blocks per position (u32, for the scan)
__global__ void __launch_bounds__(256) k_pool_blocks(uint32_t N, uint8_t *code, const uint32_t *E, const uint16_t *lp,
                                                     const uint16_t *ln, const PoolSlot *tab, uint32_t mask,
                                                     uint32_t *blk) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    uint32_t c = code[p];
    if (c == 2) {
        const unsigned long long key = (unsigned long long)E[p] << 16 | max(lp[p], ln[p]);
        uint32_t h = pool_hash(key, mask);
        while (tab[h].key != key) h = (h + 1) & mask;
        c = tab[h].min == p ? 3 : 1;
        code[p] = (uint8_t)c;
    }
    blk[p] = c == 1 ? 8u : c == 3 ? 16u : 0u;
}

// C[b] = the blocks before the end of the b-th 64-position block (P at 64b + 63)
__global__ void __launch_bounds__(256) k_pool_coarse(uint32_t N, const uint32_t *P, uint32_t *C) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if ((uint64_t)b * 64 >= N) return;
    C[b] = P[min(b * 64 + 63, N - 1)];
}

// One wave per emulating shard: the pool state from the chunk's root node on, boundary by
// boundary.  A pool boundary is the first leaf whose pattern does not fit the open pool:
// the wave keeps 64 coarse prefix values (4,096 positions) in registers, finds the block
// holding the boundary by one ballot, then its leaf with one 64-position load, and
// resolves the leaf's [5, 3] / [5, 5, 3, 3] charges.  The 2,048th pool opened inside doc g
// rotates the chunk before doc g + 1 (PiXiuCtrl.cpp:13); the window's doc count never
// reaches 65,535 (the host rotates slot-full chunks between rounds).
__global__ void __launch_bounds__(64) k_pool_scan(uint32_t nshards, const PsaShard *shards, const PsaDoc *docs,
                                                  const uint32_t *P, const uint32_t *C, uint32_t N, PsaPoolOut *out) {
    const uint32_t s = blockIdx.x;
    if (s >= nshards) return;
    const uint32_t lane = lane_id();
    const PsaShard sh = shards[s];
    PsaPoolOut o{kNone, 0, 0, 0};
    if (sh.pools && sh.ndocs) {
        auto S = [&](uint32_t x) { return x ? P[x - 1] : 0u; };  // blocks before position x
        const uint32_t start = docs[sh.doc0].start, endp = sh.base + sh.len;
        int32_t pools = 1, used = kNodeBlocks;  // the root (SuffixTree::init_prop)
        uint32_t cur = start, base = S(start);
        const uint32_t send = S(endp);
        uint32_t cw = kNone, cv = 0;  // coarse window: blocks [cw, cw + 64)
        uint32_t k_last = kNone;
        while (pools < kRotatePools && (uint32_t)used + (send - base) > (uint32_t)kPoolBlocks) {
            const uint32_t cap = (uint32_t)(kPoolBlocks - used);
            // the block holding the boundary: first b >= cur / 64 with C[b] - base > cap
            uint32_t b = cur >> 6;
            for (;;) {
                if (cw == kNone || b < cw || b >= cw + 64) {
                    cw = b;
                    const uint32_t bi = cw + lane;
                    cv = (uint64_t)bi * 64 < N ? C[bi] : 0xffffffffu;
                }
                const uint64_t m = __ballot(cw + lane >= b && ((uint64_t)(cw + lane) * 64 >= N || cv - base > cap));
                if (m) {
                    b = cw + (uint32_t)__ffsll((long long)m) - 1u;
                    break;
                }
                b = cw + 64;
            }
            const uint32_t x = b * 64 + lane;
            const uint64_t mk = __ballot(x >= cur && x < endp && P[x] - base > cap);
            const uint32_t k = mk ? b * 64 + (uint32_t)__ffsll((long long)mk) - 1u : endp - 1u;  // (mk != 0)
            const uint32_t sk = S(k);
            int32_t u = used + (int32_t)(sk - base);
            const bool split = P[k] - sk == 16u;
            const int32_t ch[4] = {kNodeBlocks, split ? kNodeBlocks : kEdgeBlocks, kEdgeBlocks, kEdgeBlocks};
            for (int i = 0; i < (split ? 4 : 2); ++i) {
                if (u + ch[i] > kPoolBlocks) {
                    ++pools;
                    u = ch[i];
                } else {
                    u += ch[i];
                }
            }
            used = u;
            cur = k + 1;
            base = P[k];
            k_last = k;
        }
        if (pools >= kRotatePools) {
            // the doc holding the 2,048th pool's first charge: rotation before the next one
            uint32_t lo = sh.doc0, hi = sh.doc0 + sh.ndocs;  // docs[lo].start <= k_last < docs[hi].start
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (docs[mid].start <= k_last) lo = mid;
                else hi = mid;
            }
            o.rot_doc = lo + 1;
        } else {
            used += (int32_t)(send - base);
        }
        o.pools = pools;
        o.used = used;
    }
    if (lane == 0) out[s] = o;
}

struct Max {
    PSA_DEV uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};

}  // namespace

#define PSA_CHECK(x)                         \
    do {                                     \
        hipError_t e_ = (x);                 \
        if (e_ != hipSuccess) return e_;     \
    } while (0)

// Runs the pipeline; messages land in every new doc's msg array, the new records' chunk /
// slot / status in rec_*, and shard_flag[k] (device, zeroed by the caller) is set for shards
// whose stream may differ from the reference's (walk them with k_gst_encode instead).
// With any_pools, the shards marked `pools` get the MemPool emulation: pool_out[k] (device)
// says where shard k's live chunk rotates inside this window (see k_pool_scan).
hipError_t psa_run(hipStream_t s, const PsaAlloc &A, uint32_t ndocs, const PsaDoc *docs, uint32_t nshards,
                   const PsaShard *shards, uint32_t N, uint32_t *rec_chunk, uint32_t *rec_idx, uint32_t *rec_status,
                   uint32_t *shard_flag, bool any_pools, PsaPoolOut *pool_out, PsaStats *st) {
    if (!N || !ndocs) return hipSuccess;
    auto get = [&](uint64_t n) { return A.alloc(A.self, n); };
    auto put = [&](void *p, uint64_t n) { A.release(A.self, p, n); };
    hipEvent_t e0, e1, e2, e3, e4;
    PSA_CHECK(hipEventCreate(&e4));
    PSA_CHECK(hipEventCreate(&e0));
    PSA_CHECK(hipEventCreate(&e1));
    PSA_CHECK(hipEventCreate(&e2));
    PSA_CHECK(hipEventCreate(&e3));
    PSA_CHECK(hipEventRecord(e0, s));
    const uint64_t n64 = N;
    auto *G = (uint8_t *)get(n64 + 64);
    auto *pdoc = (uint32_t *)get(n64 * 4);
    auto *dist = (uint16_t *)get(n64 * 2);
    auto *rank = (uint32_t *)get(n64 * 4);
    auto *sa = (uint32_t *)get(n64 * 4);
    auto *keys = (uint64_t *)get(n64 * 8);
    auto *keys2 = (uint64_t *)get(n64 * 8);
    auto *vals = (uint32_t *)get(n64 * 4);
    auto *vals2 = (uint32_t *)get(n64 * 4);
    auto *f1 = (uint32_t *)get(n64 * 4);
    auto *f2 = (uint32_t *)get(n64 * 4);
    auto *act = (uint8_t *)get(n64);
    auto *cnt = (uint32_t *)get(64);
    PSA_CHECK(hipMemsetAsync(G + N, 0, 64, s));  // (ld8 reads up to 15 bytes past the text)
    const uint32_t tb = 256;
    auto blocks = [&](uint64_t n) { return (uint32_t)((n + tb - 1) / tb); };
    int shard_bits = 1;
    while ((1u << shard_bits) <= nshards && shard_bits < 19) ++shard_bits;
    const uint32_t syms = std::min<uint32_t>(6, (64 - shard_bits) / 9);  // 5 or 6 symbols
    k_psa_gather<<<std::min<uint32_t>((ndocs + 3) / 4, 65535u), 256, 0, s>>>(ndocs, docs, G, pdoc, dist);
    k_psa_key0<<<blocks(N), tb, 0, s>>>(N, G, pdoc, docs, dist, syms, keys, vals);
    // temp storage: the largest of sort / scan / select over N elements
    size_t t_sort = 0, t_scan = 0, t_sel = 0;
    PSA_CHECK(rocprim::radix_sort_pairs(nullptr, t_sort, keys, keys2, vals, sa, (size_t)N, 0, 64, s));
    PSA_CHECK(rocprim::inclusive_scan(nullptr, t_scan, f1, f1, (size_t)N, Max(), s));
    PSA_CHECK(rocprim::select(nullptr, t_sel, sa, act, vals, cnt, (size_t)N, s));
    size_t t_sel2 = 0, t_sel3 = 0;
    PSA_CHECK(rocprim::select(nullptr, t_sel2, rocprim::counting_iterator<uint32_t>(0), act, vals, cnt, (size_t)N, s));
    PSA_CHECK(rocprim::exclusive_scan(nullptr, t_sel3, f1, f2, 0u, (size_t)N, rocprim::plus<uint32_t>(), s));
    t_sel = std::max({t_sel, t_sel2, t_sel3});
    const size_t t_bytes = std::max({t_sort, t_scan, t_sel}) + 256;
    void *tmp = get(t_bytes);
    // stream compaction (k_cmp_*): out = the flagged values (or indices), count -> cnt[0]
    const uint64_t n_tiles = (n64 + kCmpTile - 1) / kCmpTile + 1;
    auto *tcnt = (uint32_t *)get(n_tiles * 8);
    uint32_t *toff = tcnt + n_tiles;
    auto compact = [&](const uint8_t *fl, const uint32_t *vin, uint32_t *out, uint32_t n) -> hipError_t {
        const uint32_t nt = (n + kCmpTile - 1) / kCmpTile;
        if (!nt) return hipMemsetAsync(cnt, 0, 4, s);
        k_cmp_count<<<nt, 256, 0, s>>>(n, fl, tcnt);
        size_t b = t_bytes;
        const hipError_t e = rocprim::exclusive_scan(tmp, b, tcnt, toff, 0u, (size_t)nt, rocprim::plus<uint32_t>(), s);
        if (e != hipSuccess) return e;
        k_cmp_write<<<nt, 256, 0, s>>>(n, fl, vin, toff, out);
        k_cmp_total<<<1, 1, 0, s>>>(nt, tcnt, toff, cnt);
        return hipGetLastError();
    };
    size_t tb_ = t_bytes;
    PSA_CHECK(rocprim::radix_sort_pairs(tmp, tb_, keys, keys2, vals, sa, (size_t)N, 0, 9 * syms + shard_bits, s));
    k_psa_head0<<<blocks(N), tb, 0, s>>>(N, keys2, sa, dist, syms, f1);
    tb_ = t_bytes;
    PSA_CHECK(rocprim::inclusive_scan(tmp, tb_, f1, vals2, (size_t)N, Max(), s));
    k_psa_rank0<<<blocks(N), tb, 0, s>>>(N, sa, vals2, rank, act);
    tb_ = t_bytes;
    uint32_t *alist = vals;  // active suffixes, in suffix-array order
    PSA_CHECK(compact(act, sa, alist, N));
    uint32_t m = 0;
    // (counts come back through a synchronous copy after the stream drained: no async
    // copy into pageable memory, see px_runtime.cpp d2h)
    PSA_CHECK(hipStreamSynchronize(s));
    PSA_CHECK(hipMemcpy(&m, cnt, 4, hipMemcpyDeviceToHost));
    int rank_bits = 1;
    while (rank_bits < 32 && (1ull << rank_bits) <= n64) ++rank_bits;
    const bool verbose = [] {
        const char *v = std::getenv("PX_PSA_VERBOSE");
        return v && *v == '1';
    }();
    const bool segcheck = [] {
        const char *v = std::getenv("PX_PSA_SEGCHECK");
        return v && *v == '1';
    }();
    const bool segsort = [] {  // PX_PSA_SEGSORT=0: every doubling step through the radix sort
        const char *e = std::getenv("PX_PSA_SEGSORT");
        return !(e && e[0] == '0');
    }();
    // group starts and the three group lists (an active group has >= 2 suffixes: <= m/2 groups)
    const uint64_t half = n64 / 2 + 64;
    auto *gsl = segsort ? (uint32_t *)get(half * 12) : nullptr;
    uint32_t it = 0;
    for (uint32_t h = syms; m > 0; h *= 2, ++it) {
        if (st && it < 24) st->active[it] = m;
        if (it >= 20) return hipErrorUnknown;  // cannot happen: docs are <= 65,535 bytes
        k_psa_key2<<<blocks(m), tb, 0, s>>>(m, alist, rank, dist, h, keys, vals2);
        if (segsort) {
            // groups are ranges of the (suffix-array ordered) keys: sort each where it lies
            k_seg_flag<<<blocks(m), tb, 0, s>>>(m, keys, act);
            tb_ = t_bytes;
            PSA_CHECK(compact(act, nullptr, gsl, m));
            PSA_CHECK(hipStreamSynchronize(s));
            uint32_t ng = 0;
            PSA_CHECK(hipMemcpy(&ng, cnt, 4, hipMemcpyDeviceToHost));
            uint32_t *lists = gsl + half;
            const uint32_t nbk = blocks(ng);
            uint32_t *hist = gsl + 2 * half, *offs = hist + (uint64_t)kSegClasses * nbk;
            k_seg_hist<<<nbk, tb, 0, s>>>(ng, gsl, m, nbk, hist);
            tb_ = t_bytes;
            PSA_CHECK(rocprim::exclusive_scan(tmp, tb_, hist, offs, 0u, (size_t)kSegClasses * nbk, rocprim::plus<uint32_t>(), s));
            k_seg_part<<<nbk, tb, 0, s>>>(ng, gsl, m, nbk, offs, lists);
            k_seg_bounds<<<1, 64, 0, s>>>(nbk, offs, ng, cnt + 1);
            PSA_CHECK(hipStreamSynchronize(s));
            uint32_t cb[kSegClasses + 1] = {};
            PSA_CHECK(hipMemcpy(cb, cnt + 1, sizeof cb, hipMemcpyDeviceToHost));
            uint32_t c8[kSegClasses];
            uint32_t *lc[kSegClasses];
            for (int c = 0; c < kSegClasses; ++c) {
                c8[c] = cb[c + 1] - cb[c];
                lc[c] = lists + cb[c];
            }
            if (verbose)
                fprintf(stderr, "psa: step %u h=%u m=%u groups=%u (<=2..64: %u %u %u %u %u %u, <=%u: %u, larger: %u)\n",
                        it, h, m, ng, c8[0], c8[1], c8[2], c8[3], c8[4], c8[5], kSegBlock, c8[6], c8[7]);
            auto grid = [&](uint32_t n, uint32_t per_wave) {
                return std::min<uint32_t>((n + 4 * per_wave - 1) / (4 * per_wave), 1u << 16);
            };
            if (c8[0]) k_seg_sortS<2><<<grid(c8[0], 32), 256, 0, s>>>(c8[0], lc[0], gsl, ng, m, keys, vals2, keys2, f2);
            if (c8[1]) k_seg_sortS<4><<<grid(c8[1], 16), 256, 0, s>>>(c8[1], lc[1], gsl, ng, m, keys, vals2, keys2, f2);
            if (c8[2]) k_seg_sortS<8><<<grid(c8[2], 8), 256, 0, s>>>(c8[2], lc[2], gsl, ng, m, keys, vals2, keys2, f2);
            if (c8[3]) k_seg_sortS<16><<<grid(c8[3], 4), 256, 0, s>>>(c8[3], lc[3], gsl, ng, m, keys, vals2, keys2, f2);
            if (c8[4]) k_seg_sortS<32><<<grid(c8[4], 2), 256, 0, s>>>(c8[4], lc[4], gsl, ng, m, keys, vals2, keys2, f2);
            if (c8[5]) k_seg_sortS<64><<<grid(c8[5], 1), 256, 0, s>>>(c8[5], lc[5], gsl, ng, m, keys, vals2, keys2, f2);
            if (c8[6]) k_seg_sortblk<<<c8[6], 256, 0, s>>>(lc[6], gsl, ng, m, keys, vals2, keys2, f2);
            PSA_CHECK(hipGetLastError());
            uint32_t c3[3] = {0, 0, c8[7]};
            uint32_t *lbig = lc[7];
            if (c3[2]) {
                PSA_CHECK(hipMemsetAsync(act, 0, m, s));
                k_seg_mark<<<c3[2], 256, 0, s>>>(lbig, gsl, ng, m, act);
                uint32_t *tl = f1;  // free until the group-head scan below
                tb_ = t_bytes;
                PSA_CHECK(compact(act, nullptr, tl, m));
                PSA_CHECK(hipStreamSynchronize(s));
                uint32_t ml = 0;
                PSA_CHECK(hipMemcpy(&ml, cnt, 4, hipMemcpyDeviceToHost));
                auto *ck = (uint64_t *)get((uint64_t)ml * 24 + 64);
                uint64_t *ck2 = ck + ml;
                auto *cv = (uint32_t *)(ck2 + ml), *cv2 = cv + ml;
                k_seg_gather<<<blocks(ml), tb, 0, s>>>(ml, tl, keys, vals2, ck, cv);
                tb_ = t_bytes;
                PSA_CHECK(rocprim::radix_sort_pairs(tmp, tb_, ck, ck2, cv, cv2, (size_t)ml, 0, 32 + rank_bits, s));
                k_seg_scatter<<<blocks(ml), tb, 0, s>>>(ml, tl, ck2, cv2, keys2, f2);
                PSA_CHECK(hipStreamSynchronize(s));
                put(ck, (uint64_t)ml * 24 + 64);
            }
            if (segcheck) {
                auto *k3 = (uint64_t *)get((uint64_t)m * 12 + 64);
                auto *v3 = (uint32_t *)(k3 + m);
                tb_ = t_bytes;
                PSA_CHECK(rocprim::radix_sort_pairs(tmp, tb_, keys, k3, vals2, v3, (size_t)m, 0, 32 + rank_bits, s));
                PSA_CHECK(hipMemsetAsync(cnt + 12, 0, 8, s));
                k_seg_cmp<<<blocks(m), tb, 0, s>>>(m, keys2, f2, k3, v3, cnt + 12);
                PSA_CHECK(hipStreamSynchronize(s));
                uint32_t r2[2];
                PSA_CHECK(hipMemcpy(r2, cnt + 12, 8, hipMemcpyDeviceToHost));
                if (r2[0]) {
                    uint64_t a[4], b[4];
                    uint32_t va[4], vb[4];
                    const uint32_t t0 = r2[1] > 1 ? r2[1] - 1 : 0;
                    PSA_CHECK(hipMemcpy(a, keys2 + t0, 32, hipMemcpyDeviceToHost));
                    PSA_CHECK(hipMemcpy(b, k3 + t0, 32, hipMemcpyDeviceToHost));
                    PSA_CHECK(hipMemcpy(va, f2 + t0, 16, hipMemcpyDeviceToHost));
                    PSA_CHECK(hipMemcpy(vb, v3 + t0, 16, hipMemcpyDeviceToHost));
                    fprintf(stderr, "psa segcheck step %u: %u mismatches, first at t=%u\n", it, r2[0], r2[1]);
                    for (int q = 0; q < 4; ++q)
                        fprintf(stderr, "  t=%u seg %016llx/%u radix %016llx/%u\n", t0 + q, (unsigned long long)a[q], va[q],
                                (unsigned long long)b[q], vb[q]);
                }
                put(k3, (uint64_t)m * 12 + 64);
            }
        } else {
            tb_ = t_bytes;
            PSA_CHECK(rocprim::radix_sort_pairs(tmp, tb_, keys, keys2, vals2, f2, (size_t)m, 0, 32 + rank_bits, s));
        }
        // f2 = positions in the new order; group heads f1 -> vals2, subgroup heads in the
        // (now free) unsorted key buffer: flags in its first half, scan in its second
        uint32_t *sfl = (uint32_t *)keys, *sfirst = (uint32_t *)keys + N;
        k_psa_head2<<<blocks(m), tb, 0, s>>>(m, keys2, f1, sfl);
        tb_ = t_bytes;
        PSA_CHECK(rocprim::inclusive_scan(tmp, tb_, f1, vals2, (size_t)m, Max(), s));
        tb_ = t_bytes;
        PSA_CHECK(rocprim::inclusive_scan(tmp, tb_, sfl, sfirst, (size_t)m, Max(), s));
        k_psa_rank2<<<blocks(m), tb, 0, s>>>(m, keys2, f2, vals2, sfirst, sa, rank, act);
        tb_ = t_bytes;
        PSA_CHECK(compact(act, f2, alist, m));
        PSA_CHECK(hipStreamSynchronize(s));
        PSA_CHECK(hipMemcpy(&m, cnt, 4, hipMemcpyDeviceToHost));
    }
    if (st) st->iterations = it;
    put(keys2, n64 * 8);
    put(vals2, n64 * 4);
    put(act, n64);
    if (gsl) put(gsl, half * 12);
    put(tcnt, n_tiles * 8);
    put(tmp, t_bytes);
    PSA_CHECK(hipEventRecord(e1, s));
    // ---- nearest smaller positions in suffix-array order (min tree over sa)
    MinTree t{};
    t.lvl[0] = sa;
    t.n[0] = N;
    t.levels = 1;
    uint32_t *lv_buf = (uint32_t *)keys;  // the key buffer is free now: tree levels live in it
    uint64_t lv_off = 0;
    while (t.n[t.levels - 1] > 1 && t.levels < 8) {
        const uint32_t nin = t.n[t.levels - 1];
        const uint32_t nout = (nin + 63) / 64;
        uint32_t *out = lv_buf + lv_off;
        lv_off += nout;
        k_psa_minlvl<<<(nout + 3) / 4, 256, 0, s>>>(nin, t.lvl[t.levels - 1], nout, out);
        t.lvl[t.levels] = out;
        t.n[t.levels] = nout;
        ++t.levels;
    }
    uint32_t *psvp = f1, *nsvp = f2;
    {
        auto *links = (uint2 *)get(n64 * 8);
        k_psa_ansv<<<(uint32_t)((n64 + 255) / 256), 256, 0, s>>>(N, t, shards, nshards, links);
        k_psa_links_text<<<blocks(N), tb, 0, s>>>(N, rank, links, psvp, nsvp);
        put(links, n64 * 8);  // (stream-ordered reuse)
    }
    auto *lcp_p = (uint16_t *)rank;  // ranks are no longer needed: two u16 arrays in their place
    auto *lcp_n = (uint16_t *)get(n64 * 2);
    const uint32_t lsp = lce_span(n64);
    k_psa_lce<<<blocks((n64 + lsp - 1) / lsp), tb, 0, s>>>(N, (const uint64_t *)G, dist, psvp, nsvp, lcp_p, lcp_n, lsp);
    PSA_CHECK(hipEventRecord(e2, s));
    if (verbose) {
        PSA_CHECK(hipStreamSynchronize(s));
        fprintf(stderr, "psa: links + lcp done\n");
    }
    // ---- messages
    k_psa_msg0<<<blocks(N), tb, 0, s>>>(N, pdoc, docs, lcp_p, lcp_n);
    k_psa_runs<<<blocks(N), tb, 0, s>>>(N, G, pdoc, docs, dist, psvp, nsvp, lcp_p, lcp_n, shard_flag);
    k_psa_place<<<blocks(ndocs), tb, 0, s>>>(ndocs, docs, shards, rec_chunk, rec_idx, rec_status);
    PSA_CHECK(hipEventRecord(e3, s));
    if (verbose) {
        PSA_CHECK(hipStreamSynchronize(s));
        fprintf(stderr, "psa: messages done\n");
    }
    if (any_pools) {  // ---- MemPool emulation (rotation points)
        auto *code = (uint8_t *)get(n64 + 64);
        auto *E = (uint32_t *)keys, *blk = (uint32_t *)keys + N;  // the key buffer is free
        uint32_t *P = vals;
        PSA_CHECK(hipMemsetAsync(cnt + 14, 0, 4, s));
        auto *rec = (LinkRec *)get(n64 * sizeof(LinkRec));
        k_pool_pack<<<blocks(N), tb, 0, s>>>(N, psvp, nsvp, lcp_p, lcp_n, dist, rec);
        k_pool_leaf<<<blocks(N), tb, 0, s>>>(N, G, pdoc, docs, shards, rec, code, E, cnt + 14);
        put(rec, n64 * sizeof(LinkRec));  // (stream-ordered: the heap hands it out again only later)
        // the candidate table: 2x the candidates, read back for big windows; a small window
        // (one chunk, the single instance's rounds) sizes it from N and skips the round trip
        uint32_t nc = 0;
        uint64_t cap = 1024;
        const bool small_n = N <= (1u << 26);
        const bool pv = [] {
            const char *v = std::getenv("PX_PSA_VERBOSE");
            return v && *v == '1';
        }();
        if (!small_n || pv) {
            PSA_CHECK(hipStreamSynchronize(s));
            PSA_CHECK(hipMemcpy(&nc, cnt + 14, 4, hipMemcpyDeviceToHost));
            if (pv) fprintf(stderr, "psa pools: %u split candidates\n", nc);
        }
        while (cap < 2ull * (small_n ? N : nc)) cap <<= 1;
        auto *tab = (PoolSlot *)get(cap * sizeof(PoolSlot));
        PSA_CHECK(hipMemsetAsync(tab, 0xff, cap * sizeof(PoolSlot), s));
        const uint32_t mask = (uint32_t)(cap - 1);
        k_pool_insert<<<blocks(N), tb, 0, s>>>(N, code, E, lcp_p, lcp_n, tab, mask);
        if (pv) {
            PSA_CHECK(hipStreamSynchronize(s));
            fprintf(stderr, "psa pools: inserted (table %llu slots)\n", (unsigned long long)cap);
        }
        k_pool_blocks<<<blocks(N), tb, 0, s>>>(N, code, E, lcp_p, lcp_n, tab, mask, blk);
        size_t tsz = 0;
        PSA_CHECK(rocprim::inclusive_scan(nullptr, tsz, blk, P, (size_t)N, rocprim::plus<uint32_t>(), s));
        void *tmp2 = get(tsz + 256);
        PSA_CHECK(rocprim::inclusive_scan(tmp2, tsz, blk, P, (size_t)N, rocprim::plus<uint32_t>(), s));
        if (pv) {
            PSA_CHECK(hipStreamSynchronize(s));
            fprintf(stderr, "psa pools: blocks scanned\n");
        }
        auto *C = (uint32_t *)get(n64 / 64 * 4 + 256);
        k_pool_coarse<<<blocks((N + 63) / 64), tb, 0, s>>>(N, P, C);
        k_pool_scan<<<nshards, 64, 0, s>>>(nshards, shards, docs, P, C, N, pool_out);
        put(C, n64 / 64 * 4 + 256);
        PSA_CHECK(hipGetLastError());
        put(tmp2, tsz + 256);  // (stream-ordered reuse, as above)
        put(tab, cap * sizeof(PoolSlot));
        put(code, n64 + 64);
    }
    PSA_CHECK(hipEventRecord(e4, s));
    PSA_CHECK(hipEventSynchronize(e4));
    if (any_pools && st) PSA_CHECK(hipMemcpy(&st->candidates, cnt + 14, 4, hipMemcpyDeviceToHost));
    if (st) {
        PSA_CHECK(hipEventElapsedTime(&st->ms_pool, e3, e4));
        PSA_CHECK(hipEventElapsedTime(&st->ms_sort, e0, e1));
        PSA_CHECK(hipEventElapsedTime(&st->ms_lcp, e1, e2));
        PSA_CHECK(hipEventElapsedTime(&st->ms_msg, e2, e3));
        if (const char *v = std::getenv("PX_PSA_VERBOSE"); v && *v == '1') {
            fprintf(stderr, "psa: N=%u docs=%u shards=%u syms=%u sort %.2f ms, links+lcp %.2f ms, msgs %.2f ms; active:",
                    N, ndocs, nshards, syms, st->ms_sort, st->ms_lcp, st->ms_msg);
            for (uint32_t k = 0; k < it && k < 24; ++k) fprintf(stderr, " %u", st->active[k]);
            fprintf(stderr, "\n");
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipEventDestroy(e2);
    (void)hipEventDestroy(e3);
    (void)hipEventDestroy(e4);
    put(lcp_n, n64 * 2);
    put(dist, n64 * 2);
    put(G, n64 + 64);
    put(pdoc, n64 * 4);
    put(rank, n64 * 4);
    put(sa, n64 * 4);
    put(keys, n64 * 8);
    put(vals, n64 * 4);
    put(f1, n64 * 4);
    put(f2, n64 * 4);
    put(cnt, 64);
    return hipGetLastError();
}

}  // namespace px
