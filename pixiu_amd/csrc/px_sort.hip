// px_sort.hip — the suffix-array pass's sorts and scans, hand-written for gfx950.
//
// seg_sort_pairs: stable LSD radix sort of (u64 key, u32 value) pairs inside segments
// (the PSA shards of a round for the first suffix sort, the big groups of a doubling
// step).  Every pass is one "onesweep" launch over tiles of 4,096 elements of ONE
// segment: a tile ranks its elements per digit in LDS (wave ballots match equal digits;
// each wave keeps its own running counts, so ranking needs no barrier), publishes its
// per-digit counts, looks back over the earlier tiles of its segment for their running
// totals (decoupled look-back: count and flag in one word, agent-scope atomic stores and
// loads, so a flag is seen across XCDs), stages the tile in LDS in digit order and writes
// it out in runs, so consecutive lanes store consecutive addresses of one digit's run.
// The per-segment digit totals of every pass come from one histogram launch before the
// first pass.  Keys never carry the segment id: a segment's elements stay inside its
// range, which is what the rocPRIM sort over (shard | key) this replaces could not do.
//
// The first suffix sort's keys (6 symbols of 9 bits: byte + 1, 0 past the doc end;
// px_psa.hip k_psa_key0's layout) are computed from the text by the histogram and the
// first pass, so no key array is written before the sort.
//
// scan_u32: inclusive max / min / plus scans (forward or reverse) as reduce -> scan of
// block partials -> apply.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "px_route.h"
#include "px_sort.h"

namespace px {

namespace {

#define SD __device__ __forceinline__
constexpr uint32_t kThreads = 256, kItems = PX_SORT_ITEMS, kWaves = kThreads / 64;
static_assert(kThreads * kItems == kSortTile, "tile = threads x items");
constexpr uint32_t kMaxPasses = kRouteMaxPasses;
constexpr uint32_t kHistTiles = 16;       // tiles per histogram workgroup, at most (fewer for small sorts)
constexpr uint32_t kHistGroups = 1024;    // histogram workgroups a sort aims for
constexpr uint32_t kFlagAgg = 1u << 30, kFlagIncl = 2u << 30, kCountMask = (1u << 30) - 1u;
constexpr uint32_t kSpinBound = 1u << 20;  // look-back polls before a tile gives up (cannot happen)

SD uint32_t lane_id() { return threadIdx.x & 63u; }
SD uint64_t lanes_below() { return (1ull << lane_id()) - 1ull; }

// global-address-space views: a flat access waits for every outstanding memory AND LDS
// operation of the wave, which serialises the loads against the ranking's LDS traffic
#define PX_GAS __attribute__((address_space(1)))
typedef const PX_GAS uint64_t gcu64;
typedef const PX_GAS uint32_t gcu32;
typedef const PX_GAS uint16_t gcu16;
typedef PX_GAS uint64_t gu64;
typedef PX_GAS uint32_t gu32;

// the first suffix sort's key of text position p (k_psa_key0's layout without the shard):
// 8 text bytes by two aligned 8-byte loads and a funnel shift (G is 8-byte aligned and
// padded), then `syms` symbols of 9 bits; the doubling reach above them (px_sort.h kDlShift)
SD uint64_t text_key(const uint8_t *G, const uint16_t *dist, uint32_t p, uint32_t syms) {
    gcu64 *G8 = (gcu64 *)G;
    const uint32_t w = p >> 3, sh = (p & 7u) * 8u;
    uint64_t x = G8[w];
    if (sh) x = (x >> sh) | (G8[w + 1] << (64u - sh));
    const uint32_t left = ((gcu16 *)dist)[p];
    uint64_t k = 0;
    for (uint32_t s = 0; s < syms; ++s) k = k << 9 | (s < left ? ((x >> (8 * s)) & 0xffu) + 1u : 0u);
    // steps k < 15 with (syms << k) < left: 2^k <= (left - 1) / syms, i.e. that quotient's bit length
    const uint32_t q = left > syms ? (left - 1u) / syms : 0u;
    const uint32_t dl = min(15u, 32u - (uint32_t)__clz(q));
    return k | (uint64_t)dl << kDlShift;
}

// the same key from a tile's text staged in LDS (tw: the tile's 8-byte text words from
// word w0 on): no per-element global text loads (two 8-byte loads per element made the first
// pass address-bound: 8.3 ms against 5.6 for the passes that read keys)
SD uint64_t text_key_lds(const uint64_t *tw, uint32_t w0, const uint16_t *dist, uint32_t p, uint32_t syms) {
    const uint32_t w = (p >> 3) - w0, sh = (p & 7u) * 8u;
    uint64_t x = tw[w];
    if (sh) x = (x >> sh) | (tw[w + 1] << (64u - sh));
    const uint32_t left = ((gcu16 *)dist)[p];
    uint64_t k = 0;
    for (uint32_t s = 0; s < syms; ++s) k = k << 9 | (s < left ? ((x >> (8 * s)) & 0xffu) + 1u : 0u);
    const uint32_t q = left > syms ? (left - 1u) / syms : 0u;
    const uint32_t dl = min(15u, 32u - (uint32_t)__clz(q));
    return k | (uint64_t)dl << kDlShift;
}
// words of text a tile of kSortTile positions needs (its first position's word .. 8 bytes past
// its last): 4096 / 8 + 2
constexpr uint32_t kTileWords = kSortTile / 8 + 2;
// stage the text words [w0, w0 + nw) of G (8-byte aligned, padded past its end) in tw
SD void stage_text(uint64_t *tw, const uint8_t *G, uint32_t w0, uint32_t nw) {
    gcu64 *G8 = (gcu64 *)G;
    for (uint32_t i = threadIdx.x; i < nw; i += kThreads) tw[i] = G8[w0 + i];
}

// lanes (of `valid`) holding the same RB-bit digit as this lane
template <int RB>
SD uint64_t match_digit(uint32_t d, uint64_t valid) {
    uint64_t m = valid;
#pragma unroll
    for (int b = 0; b < RB; ++b) {
        const uint64_t x = __ballot((d >> b) & 1u);
        m &= ((d >> b) & 1u) ? x : ~x;
    }
    return m;
}

// exclusive scan of one value per thread over the workgroup (256 threads); total -> *tot
SD uint32_t block_excl_scan(uint32_t v, uint32_t *red, uint32_t *tot) {
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t x = v;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) red[w] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t i = 0; i < kWaves; ++i) {
        before += i < w ? red[i] : 0u;
        all += red[i];
    }
    __syncthreads();  // (red is reused by the caller's next scan)
    if (tot) *tot = all;
    return before + x - v;
}

// ---------------------------------------------------------------- histogram
// per segment and pass, the digit counts of its elements (one workgroup per `tpw` <= kHistTiles
// tiles; LDS counts flushed to the segment's global counts when the segment changes)
template <int RB, bool TEXT>
__global__ void __launch_bounds__(kThreads) k_seg_hist(const SegTile *tiles, uint32_t ntiles, uint32_t tpw, const uint64_t *kin,
                                                       const uint8_t *G, const uint16_t *dist, uint32_t syms,
                                                       uint32_t passes, uint32_t *ghist) {
    constexpr uint32_t BINS = 1u << RB;
    __shared__ uint32_t h[kMaxPasses * BINS];
    const uint32_t t0 = blockIdx.x * tpw, t1 = min(ntiles, t0 + tpw);
    for (uint32_t i = threadIdx.x; i < passes * BINS; i += kThreads) h[i] = 0;
    __syncthreads();
    uint32_t seg = tiles[t0].seg;
    auto flush = [&]() {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < passes * BINS; i += kThreads) {
            if (h[i]) atomicAdd(ghist + (uint64_t)seg * passes * BINS + i, h[i]);
            h[i] = 0;
        }
        __syncthreads();
    };
    for (uint32_t t = t0; t < t1; ++t) {
        const SegTile T = tiles[t];
        if (T.seg != seg) {  // (workgroup-uniform)
            flush();
            seg = T.seg;
        }
        for (uint32_t j0 = 0; j0 < T.count; j0 += kThreads) {
            const uint32_t j = j0 + threadIdx.x;
            const bool ok = j < T.count;
            uint64_t k = 0;
            if (ok) k = TEXT ? text_key(G, dist, T.start + j, syms) : ((gcu64 *)kin)[T.start + j];
            const uint64_t valid = __ballot(ok);
            for (uint32_t p = 0; p < passes; ++p) {
                const uint32_t d = (uint32_t)(k >> (RB * p)) & (BINS - 1u);
                const uint64_t m = match_digit<RB>(d, valid);
                if (ok && (m & lanes_below()) == 0) atomicAdd(&h[p * BINS + d], (uint32_t)__popcll(m));
            }
        }
    }
    flush();
}

// The first suffix sort's histograms from one symbol histogram: pass p's digit of suffix j
// is its symbol s = syms-1-p, i.e. the first symbol of suffix j+s while j+s stays in j's
// doc, else 0 (past the doc end).  So pass p's counts = the first-symbol counts (pass
// syms-1's own), less the symbols at offsets < s of every doc, plus one 0 per suffix within
// s of its doc's end.  One match per element instead of `syms`; a doc's first thread (the
// segment's first position, or one after a doc's last, dist == 1) takes its first offsets'
// corrections from the 8 text bytes it loaded, every suffix near its doc's end its zeros.
// (Counts wrap: the corrections are subtracted in u32 and the sums are exact.)
__global__ void __launch_bounds__(kThreads) k_seg_hist_text(const SegTile *tiles, uint32_t ntiles, uint32_t tpw, const uint8_t *G,
                                                            const uint16_t *dist, uint32_t syms, uint32_t *ghist) {
    constexpr uint32_t BINS = 512;
    __shared__ uint32_t h[kMaxPasses * BINS];  // pass syms-1: the first-symbol counts; others: corrections
    __shared__ uint64_t tw[kTileWords];         // the tile's text
    const uint32_t t0 = blockIdx.x * tpw, t1 = min(ntiles, t0 + tpw), top = syms - 1;
    for (uint32_t i = threadIdx.x; i < syms * BINS; i += kThreads) h[i] = 0;
    __syncthreads();
    uint32_t seg = tiles[t0].seg;
    auto flush = [&]() {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < syms * BINS; i += kThreads) {
            const uint32_t p = i / BINS, v = i % BINS;
            const uint32_t c = p == top ? h[i] : h[i] + h[top * BINS + v];
            if (c) atomicAdd(ghist + (uint64_t)seg * syms * BINS + i, c);
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < syms * BINS; i += kThreads) h[i] = 0;
        __syncthreads();
    };
    for (uint32_t t = t0; t < t1; ++t) {
        const SegTile T = tiles[t];
        if (T.seg != seg) {  // (workgroup-uniform)
            flush();
            seg = T.seg;
        }
        const uint32_t tw0 = T.start >> 3;
        __syncthreads();  // (the previous tile's text is read)
        stage_text(tw, G, tw0, min(kTileWords, ((T.start + T.count + 8u) >> 3) + 1u - tw0));
        __syncthreads();
        for (uint32_t j0 = 0; j0 < T.count; j0 += kThreads) {
            const uint32_t j = j0 + threadIdx.x;
            const bool ok = j < T.count;
            uint32_t d = 0;
            if (ok) {
                const uint32_t pos = T.start + j, w = (pos >> 3) - tw0, sh = (pos & 7u) * 8u;
                uint64_t x = tw[w];
                if (sh) x = (x >> sh) | (tw[w + 1] << (64u - sh));
                const uint32_t left = ((gcu16 *)dist)[pos];  // (>= 1)
                d = (uint32_t)(x & 0xffu) + 1u;
                for (uint32_t s = left; s <= top; ++s) atomicAdd(&h[(top - s) * BINS], 1u);  // past the doc end
                const bool doc0 = (T.first && j == 0) || ((gcu16 *)dist)[pos - 1] == 1;
                if (doc0) {
                    for (uint32_t o = 0; o + 1 <= top && o < left; ++o) {
                        const uint32_t v = (uint32_t)((x >> (8 * o)) & 0xffu) + 1u;
                        for (uint32_t s = o + 1; s <= top; ++s) atomicSub(&h[(top - s) * BINS + v], 1u);
                    }
                }
            }
            const uint64_t m = match_digit<9>(d, __ballot(ok));
            if (ok && (m & lanes_below()) == 0) atomicAdd(&h[top * BINS + d], (uint32_t)__popcll(m));
        }
    }
    flush();
}

// the tile table on the device: tiles before each segment (one workgroup), then one
// thread per tile finds its segment by a binary search over that prefix
__global__ void __launch_bounds__(1024) k_seg_tpre(uint32_t nseg, const uint32_t *len, uint32_t *pre) {
    __shared__ uint32_t red[16];
    const uint32_t per = (nseg + 1023) / 1024, a = threadIdx.x * per, e = min(nseg, a + per);
    uint32_t acc = 0;
    for (uint32_t g = a; g < e; ++g) acc += (len[g] + kSortTile - 1) / kSortTile;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t x = acc;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) red[w] = x;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t i = 0; i < w; ++i) before += red[i];
    uint32_t run = before + x - acc;
    for (uint32_t g = a; g < e; ++g) {
        pre[g] = run;
        run += (len[g] + kSortTile - 1) / kSortTile;
    }
    if (threadIdx.x == 1023) pre[nseg] = before + x;
}
__global__ void __launch_bounds__(256) k_seg_tfill(uint32_t nt, uint32_t nseg, const uint32_t *start, const uint32_t *len,
                                                   const uint32_t *pre, SegTile *tiles) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nt) return;
    uint32_t lo = 0, hi = nseg;  // the last segment g with pre[g] <= t
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= t) lo = mid;
        else hi = mid;
    }
    const uint32_t o = (t - pre[lo]) * kSortTile;
    tiles[t] = SegTile{start[lo] + o, min(kSortTile, len[lo] - o), lo, o == 0 ? 1u : 0u};
}

// where each digit's run of each segment starts: the segment's start + the exclusive
// prefix of its digit counts (one workgroup per segment and pass)
template <int RB>
__global__ void __launch_bounds__(kThreads) k_seg_base(const uint32_t *ghist, const uint32_t *seg_start,
                                                       uint32_t passes, uint32_t *base) {
    constexpr uint32_t BINS = 1u << RB, BPT = BINS / kThreads;
    __shared__ uint32_t red[kWaves];
    const uint32_t sp = blockIdx.x, seg = sp / passes;
    const uint32_t *hp = ghist + (uint64_t)sp * BINS;
    uint32_t v[BPT], sum = 0;
#pragma unroll
    for (uint32_t i = 0; i < BPT; ++i) {
        v[i] = hp[threadIdx.x * BPT + i];
        sum += v[i];
    }
    uint32_t run = seg_start[seg] + block_excl_scan(sum, red, nullptr);
#pragma unroll
    for (uint32_t i = 0; i < BPT; ++i) {
        base[(uint64_t)sp * BINS + threadIdx.x * BPT + i] = run;
        run += v[i];
    }
}

// ---------------------------------------------------------------- one radix pass
template <int RB, bool TEXT>
#ifndef PX_SORT_WPE
#define PX_SORT_WPE 1
#endif
__global__ void __launch_bounds__(kThreads, PX_SORT_WPE) k_seg_pass(const SegTile *tiles, uint32_t *tile_ctr, const uint64_t *kin_,
                                                       const uint32_t *vin_, uint64_t *kout_, uint32_t *vout_,
                                                       uint32_t pass, uint32_t passes, const uint32_t *base,
                                                       uint32_t *status, const uint8_t *G, const uint16_t *dist,
                                                       uint32_t syms, uint32_t *err, uint32_t *status_next) {
    constexpr uint32_t BINS = 1u << RB, BPT = BINS / kThreads;
    // (the tile number and the scan's partials live in s_dst's first words, which are written only
    // after both are spent)
    __shared__ uint16_t wh[kWaves][BINS];  // per wave: running count, then the wave's offset in the tile
    __shared__ uint32_t s_excl[BINS];      // tile-local start of each digit's run
    __shared__ uint32_t s_dst[BINS];       // global position of that run's first element
    __shared__ uint64_t stage[kSortTile];  // the tile in digit order: keys, then values
    __shared__ uint16_t sdig[kSortTile];   // and each staged element's digit
    uint32_t &s_tile = s_dst[0];
    uint32_t *red = s_dst + 4;
    gcu64 *kin = (gcu64 *)kin_;
    gcu32 *vin = (gcu32 *)vin_;
    gu64 *kout = (gu64 *)kout_;
    gu32 *vout = (gu32 *)vout_;
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6, shift = RB * pass;
    if (threadIdx.x == 0) s_tile = atomicAdd(tile_ctr, 1u);  // tiles start in order: look-back never waits on a later one
    for (uint32_t i = threadIdx.x; i < kWaves * BINS; i += kThreads) (&wh[0][0])[i] = 0;
    __syncthreads();
    const uint32_t t = s_tile;
    const SegTile T = tiles[t];
    // the next pass's look-back words of this tile cleared here (that buffer was the previous
    // pass's, which is complete): one memset per sort instead of one per pass
    if (status_next)
        for (uint32_t i = threadIdx.x; i < BINS; i += kThreads) ((gu32 *)status_next)[(uint64_t)t * BINS + i] = 0;
    // (the first pass: the tile's text in LDS, in the stage buffer's room until the ranking)
    const uint32_t tw0 = T.start >> 3;
    if (TEXT) {
        stage_text(&stage[0], G, tw0, min(kTileWords, ((T.start + T.count + 8u) >> 3) + 1u - tw0));
        __syncthreads();
    }
    // ---- load: wave w takes elements [w * 1024, (w + 1) * 1024) of the tile, 64 at a time
    uint64_t k[kItems];
    uint32_t v[kItems];
    uint16_t r[kItems];
    const uint32_t j0 = w * (kItems * 64) + lane;
#pragma unroll
    for (uint32_t it = 0; it < kItems; ++it) {
        const uint32_t j = j0 + it * 64;
        k[it] = 0;
        v[it] = 0;
        if (j < T.count) {
            if (TEXT) {
                k[it] = text_key_lds(&stage[0], tw0, dist, T.start + j, syms);
                v[it] = T.start + j;
            } else {
                k[it] = kin[T.start + j];
                v[it] = vin[T.start + j];
            }
        }
    }
    // ---- rank: each wave counts its own digits (no barrier inside)
#pragma unroll
    for (uint32_t it = 0; it < kItems; ++it) {
        const bool ok = j0 + it * 64 < T.count;
        const uint32_t d = (uint32_t)(k[it] >> shift) & (BINS - 1u);
        const uint64_t m = match_digit<RB>(d, __ballot(ok));
        uint32_t prev = 0;
        if (ok) prev = wh[w][d];
        const uint32_t below = (uint32_t)__popcll(m & lanes_below());
        r[it] = (uint16_t)(prev + below);
        if (ok && below == 0) wh[w][d] = (uint16_t)(prev + (uint32_t)__popcll(m));
    }
    __syncthreads();
    // ---- per digit: the waves' offsets, the tile's count, its run start in the tile
    uint32_t cnt[BPT], tsum = 0;
#pragma unroll
    for (uint32_t i = 0; i < BPT; ++i) {
        const uint32_t b = threadIdx.x * BPT + i;
        uint32_t c = 0;
        for (uint32_t x = 0; x < kWaves; ++x) {
            const uint32_t y = wh[x][b];
            wh[x][b] = (uint16_t)c;
            c += y;
        }
        cnt[i] = c;
        tsum += c;
    }
    uint32_t run = block_excl_scan(tsum, red, nullptr);
#pragma unroll
    for (uint32_t i = 0; i < BPT; ++i) {
        s_excl[threadIdx.x * BPT + i] = run;
        run += cnt[i];
    }
    // ---- look-back over the earlier tiles of this segment, every digit of the thread at once
    const uint32_t *sb = base + ((uint64_t)T.seg * passes + pass) * BINS;
    uint32_t excl[BPT], done = 0, fail = 0;
#pragma unroll
    for (uint32_t i = 0; i < BPT; ++i) {
        excl[i] = 0;
        uint32_t *mine = status + (uint64_t)t * BINS + threadIdx.x * BPT + i;
        __hip_atomic_store(mine, (T.first ? kFlagIncl : kFlagAgg) | cnt[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (T.first) done |= 1u << i;
    }
    if (done != (1u << BPT) - 1u) {
        uint32_t j[BPT], spins = 0;
#pragma unroll
        for (uint32_t i = 0; i < BPT; ++i) j[i] = t - 1;
        while (done != (1u << BPT) - 1u) {
            uint32_t x[BPT];
#pragma unroll
            for (uint32_t i = 0; i < BPT; ++i)
                x[i] = (done >> i) & 1u ? 0u
                                        : __hip_atomic_load(status + (uint64_t)j[i] * BINS + threadIdx.x * BPT + i,
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool waited = false;
#pragma unroll
            for (uint32_t i = 0; i < BPT; ++i) {
                if ((done >> i) & 1u) continue;
                if ((x[i] & ~kCountMask) == 0) {
                    waited = true;
                    continue;
                }
                excl[i] += x[i] & kCountMask;
                if ((x[i] & ~kCountMask) == kFlagIncl) done |= 1u << i;
                else --j[i];
            }
            if (waited && ++spins > kSpinBound) {
                fail = 1;
                break;
            }
        }
#pragma unroll
        for (uint32_t i = 0; i < BPT; ++i)
            __hip_atomic_store(status + (uint64_t)t * BINS + threadIdx.x * BPT + i, kFlagIncl | (excl[i] + cnt[i]),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (uint32_t i = 0; i < BPT; ++i) s_dst[threadIdx.x * BPT + i] = sb[threadIdx.x * BPT + i] + excl[i];
    if (fail) atomicOr(err, 1u);
    __syncthreads();
    // ---- stage the keys in digit order, write each digit's run to its place
    // (consecutive lanes, consecutive addresses); then the values the same way
    // (staging the values as value | digit << 32 instead of keeping sdig measured slower: the first
    // sort 43.3 -> 45.7 ms, profiles/r06e_*; without sdig the LDS would allow a fourth workgroup
    // per CU, but the registers (166 VGPRs) keep it at three)
    uint16_t at[kItems];
#pragma unroll
    for (uint32_t it = 0; it < kItems; ++it) {
        const uint32_t d = (uint32_t)(k[it] >> shift) & (BINS - 1u);
        at[it] = (uint16_t)(s_excl[d] + wh[w][d] + r[it]);
        if (j0 + it * 64 < T.count) {
            stage[at[it]] = k[it];
            sdig[at[it]] = (uint16_t)d;
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < T.count; i += kThreads) {
        const uint32_t d = sdig[i];
        kout[s_dst[d] + (i - s_excl[d])] = stage[i];
    }
    __syncthreads();
    uint32_t *sv = reinterpret_cast<uint32_t *>(&stage[0]);
#pragma unroll
    for (uint32_t it = 0; it < kItems; ++it)
        if (j0 + it * 64 < T.count) sv[at[it]] = v[it];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < T.count; i += kThreads) {
        const uint32_t d = sdig[i];
        vout[s_dst[d] + (i - s_excl[d])] = sv[i];
    }
}

// ---------------------------------------------------------------- scans
template <ScanOp OP>
SD uint32_t op_id() {
    return OP == ScanOp::kMax ? 0u : OP == ScanOp::kMin ? 0xffffffffu : 0u;
}
template <ScanOp OP>
SD uint32_t op_do(uint32_t a, uint32_t b) {
    return OP == ScanOp::kMax ? max(a, b) : OP == ScanOp::kMin ? min(a, b) : a + b;
}
constexpr uint32_t kScanItems = 16, kScanBlock = kThreads * kScanItems;  // elements per workgroup (16 per
                                                                          // thread, whatever the sort tile)

template <ScanOp OP, bool REV>
SD uint64_t scan_at(uint64_t i, uint64_t n) { return REV ? n - 1 - i : i; }

template <ScanOp OP>
SD uint32_t block_incl_scan(uint32_t x, uint32_t *red, uint32_t *all) {
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x = op_do<OP>(x, y);
    }
    if (lane == 63) red[w] = x;
    __syncthreads();
    uint32_t before = op_id<OP>(), tot = op_id<OP>();
    for (uint32_t i = 0; i < kWaves; ++i) {
        if (i < w) before = op_do<OP>(before, red[i]);
        tot = op_do<OP>(tot, red[i]);
    }
    __syncthreads();
    if (all) *all = tot;
    return op_do<OP>(before, x);
}

template <ScanOp OP, bool REV>
__global__ void __launch_bounds__(kThreads) k_scan_reduce(const uint32_t *in, uint64_t n, uint32_t *part) {
    __shared__ uint32_t red[kWaves];
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanBlock;
    uint32_t acc = op_id<OP>();
    for (uint32_t j = threadIdx.x; j < kScanBlock; j += kThreads) {
        const uint64_t i = b0 + j;
        if (i < n) acc = op_do<OP>(acc, in[scan_at<OP, REV>(i, n)]);
    }
    uint32_t all;
    (void)block_incl_scan<OP>(acc, red, &all);
    if (threadIdx.x == 0) part[blockIdx.x] = all;
}
// exclusive scan of the block partials, one workgroup
template <ScanOp OP>
__global__ void __launch_bounds__(1024) k_scan_parts(uint32_t *part, uint32_t nb) {
    __shared__ uint32_t red[16];
    const uint32_t per = (nb + 1023) / 1024, a = threadIdx.x * per, e = min(nb, a + per);
    uint32_t acc = op_id<OP>();
    for (uint32_t i = a; i < e; ++i) acc = op_do<OP>(acc, part[i]);
    // exclusive scan of acc over the 1,024 threads (16 waves)
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    uint32_t x = acc;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x = op_do<OP>(x, y);
    }
    if (lane == 63) red[w] = x;
    __syncthreads();
    uint32_t before = op_id<OP>();
    for (uint32_t i = 0; i < w; ++i) before = op_do<OP>(before, red[i]);
    uint32_t run = op_do<OP>(before, (uint32_t)__shfl_up((int)x, 1));
    if (lane == 0) run = before;
    for (uint32_t i = a; i < e; ++i) {
        const uint32_t y = part[i];
        part[i] = run;
        run = op_do<OP>(run, y);
    }
}
template <ScanOp OP, bool REV>
__global__ void __launch_bounds__(kThreads) k_scan_apply(const uint32_t *in, uint32_t *out, uint64_t n,
                                                         const uint32_t *part) {
    __shared__ uint32_t red[kWaves];
    const uint64_t b0 = (uint64_t)blockIdx.x * kScanBlock;
    // each thread: 16 consecutive elements (in scan order)
    const uint64_t i0 = b0 + (uint64_t)threadIdx.x * kScanItems;
    uint32_t x[kScanItems], acc = op_id<OP>();
#pragma unroll
    for (uint32_t j = 0; j < kScanItems; ++j) {
        const uint64_t i = i0 + j;
        x[j] = i < n ? in[scan_at<OP, REV>(i, n)] : op_id<OP>();
        acc = op_do<OP>(acc, x[j]);
    }
    const uint32_t incl = block_incl_scan<OP>(acc, red, nullptr);
    // exclusive of this thread = the block carry + the threads before it
    uint32_t run = (uint32_t)__shfl_up((int)incl, 1);
    __shared__ uint32_t last[kWaves];
    if (lane_id() == 63) last[threadIdx.x >> 6] = incl;
    __syncthreads();
    if (lane_id() == 0) run = threadIdx.x ? last[(threadIdx.x >> 6) - 1] : op_id<OP>();
    run = op_do<OP>(part[blockIdx.x], run);
#pragma unroll
    for (uint32_t j = 0; j < kScanItems; ++j) {
        const uint64_t i = i0 + j;
        run = op_do<OP>(run, x[j]);
        if (i < n) out[scan_at<OP, REV>(i, n)] = run;
    }
}

template <ScanOp OP, bool REV>
hipError_t scan_run(hipStream_t s, const SortAlloc &A, const uint32_t *in, uint32_t *out, uint64_t n) {
    if (!n) return hipSuccess;
    const uint64_t nb = (n + kScanBlock - 1) / kScanBlock;
    if (nb > 0xffffffffull) return hipErrorInvalidValue;
    auto *part = (uint32_t *)A.alloc(A.self, nb * 4 + 64);
    if (!part) return hipErrorOutOfMemory;
    k_scan_reduce<OP, REV><<<(uint32_t)nb, kThreads, 0, s>>>(in, n, part);
    k_scan_parts<OP><<<1, 1024, 0, s>>>(part, (uint32_t)nb);
    k_scan_apply<OP, REV><<<(uint32_t)nb, kThreads, 0, s>>>(in, out, n, part);
    A.release(A.self, part, nb * 4 + 64);
    return hipGetLastError();
}

}  // namespace

uint32_t seg_tile_count(const uint32_t *len, uint32_t nseg) {
    uint64_t t = 0;
    for (uint32_t g = 0; g < nseg; ++g) t += (len[g] + kSortTile - 1) / kSortTile;
    return (uint32_t)t;
}

hipError_t seg_sort_pairs(hipStream_t s, const SortAlloc &A, uint32_t nseg, uint32_t nt, const uint32_t *d_start,
                          const uint32_t *d_len, uint32_t bits, int rb, uint64_t *k0, uint32_t *v0, const uint8_t *G,
                          const uint16_t *dist, uint32_t syms, uint64_t *ka, uint32_t *va, uint64_t *kb, uint32_t *vb,
                          uint64_t *kout, uint32_t *vout, uint32_t *err) {
    if (!nt) return hipSuccess;
    if (rb != 8 && rb != 9) return hipErrorInvalidValue;
    const bool text = G != nullptr;
    const uint32_t bins = 1u << rb, passes = (bits + rb - 1) / rb;
    if (passes == 0 || passes > kMaxPasses) return hipErrorInvalidValue;
    // scratch: tiles, tiles before each segment, digit counts and run starts, tile counters,
    // look-back words
    const uint64_t b_tiles = (uint64_t)nt * sizeof(SegTile), b_pre = ((uint64_t)nseg + 1) * 4,
                   b_hist = (uint64_t)nseg * passes * bins * 4, b_status = (uint64_t)nt * bins * 4;
    const uint64_t o_pre = (b_tiles + 255) / 256 * 256, o_hist = o_pre + (b_pre + 255) / 256 * 256,
                   o_base = o_hist + (b_hist + 255) / 256 * 256, o_ctr = o_base + (b_hist + 255) / 256 * 256,
                   o_status = o_ctr + 256, o_status2 = o_status + (b_status + 255) / 256 * 256,
                   total = o_status2 + b_status + 256;
    auto *mem = (uint8_t *)A.alloc(A.self, total);
    if (!mem) return hipErrorOutOfMemory;
    auto *d_tiles = (SegTile *)mem;
    auto *d_pre = (uint32_t *)(mem + o_pre);
    auto *d_hist = (uint32_t *)(mem + o_hist);
    auto *d_base = (uint32_t *)(mem + o_base);
    auto *d_ctr = (uint32_t *)(mem + o_ctr);
    // two look-back buffers, alternating by pass: pass p clears the one pass p + 1 uses
    uint32_t *d_status2[2] = {(uint32_t *)(mem + o_status), (uint32_t *)(mem + o_status2)};
    // one memset: the digit counts, (the bases, written whole later), the tile counters and the
    // first pass's look-back words
    hipError_t e = hipMemsetAsync(d_hist, 0, o_status + b_status - o_hist, s);
    static const bool per_pass_memset = [] {  // (A/B: one memset per pass, as before)
        const char *v = std::getenv("PX_SORT_PASS_MEMSET");
        return v && *v == '1';
    }();
    if (e != hipSuccess) {
        A.release(A.self, mem, total);
        return e;
    }
    k_seg_tpre<<<1, 1024, 0, s>>>(nseg, d_len, d_pre);
    k_seg_tfill<<<(nt + 255) / 256, 256, 0, s>>>(nt, nseg, d_start, d_len, d_pre, d_tiles);
    // (a small sort -- the big groups of a single-instance round -- spreads its tiles thin:
    // 16 tiles per workgroup left ~30 workgroups, each walking 64 K elements alone)
    // (fewer, longer histogram workgroups for one-segment sorts -- to spare the flush atomics --
    // measured slower: a single-instance round's first sort 61 -> 195 us, r06w)
    const uint32_t tpw = std::max<uint32_t>(1, std::min<uint32_t>(kHistTiles, (nt + kHistGroups - 1) / kHistGroups));
    const uint32_t hb = (nt + tpw - 1) / tpw;
    // every pass's output pair (px_route.h: no pass writes a buffer it reads, for any pass count)
    BufPair route[kRouteMaxPasses];
    {
        const BufPair scratch[4] = {{ka, va}, {kb, vb}, {text ? nullptr : k0, text ? nullptr : v0}, {kout, vout}};
        if (!sort_route(passes, BufPair{text ? nullptr : k0, text ? nullptr : v0}, scratch, BufPair{kout, vout}, route)) {
            A.release(A.self, mem, total);
            return hipErrorInvalidValue;
        }
    }
#define PX_SORT_RB(RB_)                                                                                            \
    do {                                                                                                           \
        if (text && RB_ == 9 && passes == syms)                                                                    \
            k_seg_hist_text<<<hb, kThreads, 0, s>>>(d_tiles, nt, tpw, G, dist, syms, d_hist);                           \
        else if (text)                                                                                             \
            k_seg_hist<RB_, true><<<hb, kThreads, 0, s>>>(d_tiles, nt, tpw, nullptr, G, dist, syms, passes, d_hist);    \
        else                                                                                                       \
            k_seg_hist<RB_, false><<<hb, kThreads, 0, s>>>(d_tiles, nt, tpw, k0, nullptr, nullptr, 0, passes, d_hist);  \
        k_seg_base<RB_><<<nseg * passes, kThreads, 0, s>>>(d_hist, d_start, passes, d_base);                      \
        const uint64_t *ki = k0;                                                                                   \
        const uint32_t *vi = v0;                                                                                   \
        for (uint32_t p = 0; p < passes && e == hipSuccess; ++p) {                                                 \
            uint64_t *ko = (uint64_t *)route[p].k;                                                                 \
            uint32_t *vo = (uint32_t *)route[p].v;                                                                 \
            uint32_t *st = d_status2[p & 1u], *sn = p + 1 < passes ? d_status2[(p + 1) & 1u] : nullptr;          \
            if (per_pass_memset) {                                                                                 \
                st = d_status2[0];                                                                                 \
                sn = nullptr;                                                                                      \
                if (p > 0) e = hipMemsetAsync(st, 0, b_status, s);                                                 \
            }                                                                                                      \
            if (text && p == 0)                                                                                    \
                k_seg_pass<RB_, true><<<nt, kThreads, 0, s>>>(d_tiles, d_ctr + p, nullptr, nullptr, ko, vo, p,     \
                                                              passes, d_base, st, G, dist, syms, err, sn);         \
            else                                                                                                   \
                k_seg_pass<RB_, false><<<nt, kThreads, 0, s>>>(d_tiles, d_ctr + p, ki, vi, ko, vo, p, passes,      \
                                                               d_base, st, nullptr, nullptr, 0, err, sn);          \
            ki = ko;                                                                                               \
            vi = vo;                                                                                               \
            e = hipGetLastError();                                                                                 \
        }                                                                                                          \
    } while (0)
    if (rb == 9)
        PX_SORT_RB(9);
    else
        PX_SORT_RB(8);
#undef PX_SORT_RB
    A.release(A.self, mem, total);  // (stream-ordered reuse: later work on this stream only)
    return e;
}

hipError_t scan_u32(hipStream_t s, const SortAlloc &A, const uint32_t *in, uint32_t *out, uint64_t n, ScanOp op,
                    bool reverse) {
    switch (op) {
    case ScanOp::kMax: return reverse ? scan_run<ScanOp::kMax, true>(s, A, in, out, n) : scan_run<ScanOp::kMax, false>(s, A, in, out, n);
    case ScanOp::kMin: return reverse ? scan_run<ScanOp::kMin, true>(s, A, in, out, n) : scan_run<ScanOp::kMin, false>(s, A, in, out, n);
    default: return reverse ? scan_run<ScanOp::kPlus, true>(s, A, in, out, n) : scan_run<ScanOp::kPlus, false>(s, A, in, out, n);
    }
}

}  // namespace px
