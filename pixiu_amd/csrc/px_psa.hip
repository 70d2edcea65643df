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
//   first sort     6 symbols of 9 bits per suffix, a segmented radix sort inside each
//                  shard whose first pass reads the text (px_sort.hip, hand-written)
//   prefix doubling: keys (group, rank[p+h]) of unsorted suffixes only, sorted inside their
//                  groups (windows / registers / LDS; the largest by px_sort.hip's
//                  segmented sort), group heads by max-scans, ranks and SA written back
//   k_psa_minlvl / k_psa_ansv_blk   nearest smaller position left/right in SA order
//                  (a 64-ary min tree; one wave per 64 ranks, ballot descents)
//   k_psa_lce      lcp with those two neighbours, Kasai-style in text order
//                  (lcp(p) >= lcp(p-1) - 1 for both neighbours)
//   k_psa_msg0 / k_psa_runs   messages, earliest occurrences (neighbour chains), the
//                  stale-pair check; k_psa_place   chunk / slot / status per record
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include <hip/hip_runtime.h>

#include "px_common.h"
#include "px_sort.h"

namespace px {

namespace {

constexpr uint32_t kNoPos = 0xffffffffu;
constexpr uint32_t kPass = 0xffffffffu;
#define PSA_DEV __device__ __forceinline__
#define PX_GAS __attribute__((address_space(1)))

PSA_DEV uint32_t lane_id() { return threadIdx.x & 63u; }

// ---------------------------------------------------------------- text
// G = the text, pdoc = doc id and dist = bytes to the doc's end, per position.  One wave per
// slice of a doc (`slices` per doc, so that a window of a few long docs -- a single-instance
// round holds ~210 -- still spreads over the chip)
__global__ void __launch_bounds__(256) k_psa_gather(uint32_t ndocs, const PsaDoc *docs, uint32_t slices, uint8_t *G,
                                                    uint32_t *pdoc, uint16_t *dist) {
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    const uint64_t nw = (uint64_t)ndocs * slices;
    for (uint64_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); w < nw; w += waves) {
        const uint32_t g = (uint32_t)(w / slices), sl = (uint32_t)(w % slices);
        const PsaDoc d = docs[g];
        const uint32_t lo = (uint32_t)((uint64_t)d.len * sl / slices), hi = (uint32_t)((uint64_t)d.len * (sl + 1) / slices);
        const PX_GAS uint8_t *src = (const PX_GAS uint8_t *)d.src;
        for (uint32_t o = lo + lane; o < hi; o += 64) {
            G[d.start + o] = src[o];
            pdoc[d.start + o] = g;
            dist[d.start + o] = (uint16_t)(d.len - o);  // 1..65,535
        }
    }
}

// ---------------------------------------------------------------- unsorted groups
// Prefix doubling keeps the suffixes that still share their first h symbols with another
// suffix in GROUPS: a group is a range [start, start + size) of the suffix array, and
// rank[p] = the group's start for each of its suffixes.  A step sorts every group by the
// rank of the suffix h further on (0 past the doc end), rewriting sa inside the group, and
// its subgroups (equal keys) become the next step's groups.  State per suffix-array slot:
//   act[slot] = 1   the slot's suffix is in a group (still unsorted)
//   gsz[slot]       at a group's first slot: size | tag << 31, where tag = the parity of the
//                   step that sorts it (groups a step creates are invisible to that step)
//   key[slot]       this step's key, gathered by k_dbl_key before any group is sorted, so
//                   the sorters can write the new ranks directly
// Sorting by group size: <= 64 where they lie (k_dbl_win: one wave per 64-slot window sorts
// the groups starting in it), 65..kRegMax by one wave in registers, up to kMedMax by one
// workgroup in LDS, larger ones by a gathered radix sort (host-driven: only early steps).
constexpr uint32_t kWinMax = 64, kRegMax = 512, kMedMax = 4096;
constexpr uint32_t kTag = 1u << 31, kSizeMask = kTag - 1u;
constexpr int kLongClasses = 5;  // E = 2, 4, 8 (registers), LDS, big
constexpr int kBigClass = kLongClasses - 1;
struct LongLists {
    uint64_t *lst[kLongClasses];  // entry: start | size << 32
    uint32_t *cnt;                // [0..4] entries, [5] overflow flag
    uint32_t cap[kLongClasses];
};
PSA_DEV uint32_t long_class(uint32_t size) {
    return size <= 128 ? 0u : size <= 256 ? 1u : size <= kRegMax ? 2u : size <= kMedMax ? 3u : 4u;
}

// ---------------------------------------------------------------- retired groups
// A group G (slots [g, g + size)) whose members all keep one key K at a step with offset h
// -- every suffix h further on lies in the group G' that starts at slot t = K - 1 -- and
// whose G' has exactly |G| members is a shifted copy of G': the map p -> p + h is a
// bijection G -> G', the members share their first h symbols and none ends inside them, so
// G's final order is G''s, shifted by h (equal suffixes stay in position order too).  Such a
// group leaves the doubling at once instead of being re-keyed at every later step until its
// copies diverge (the templates every page of a shard repeats: ~80 M suffixes for 8 steps on
// config 3).  Its members' ranks name its entry (id | kRetired).  An entry links G to the
// slot range [T, T + size) that holds its members shifted by D (at first T = t, D = h); a
// rank read that hits a member q is answered through the link: g + (rank(q + D) - T) -- G
// mirrors the current partition of the range, so these ranks refine the current level and
// order the suffixes as the true ranks do, which is all a doubling key needs -- and so on
// through any retired group there.  When one retired group covers a link's range exactly
// (the same-step chains of a template's offsets), the link can take that group's own link
// instead (path compression while reading; pointer jumping over all entries at the end).
// After the doubling every retired member's rank read through its links is its final slot.
// (tools/proto/retire_proto.py is the CPU prototype, checked against a naive suffix sort.)
constexpr uint32_t kRetired = 1u << 31;  // (ranks are slot indices < 2^31)
constexpr uint32_t kMaxHops = 1u << 20;  // link hops of one rank read (cannot be reached: positions rise every hop)
// Entries are handed out from kRetShards counters, each on a line of its own and owning
// `per` consecutive ids (one counter for the whole launch serialised every retiring wave on
// one address: k_dbl_win went from 3 to 29 ms a step)
constexpr uint32_t kRetShards = 64, kRetStride = 32;
struct RetList {
    uint4 *ent;               // g, size, q0 (a member's position), first shift
    unsigned long long *lnk;  // T | D << 32 (64-bit atomic: read and shortened concurrently)
    uint32_t *cnt;            // [1] a link led out of range (cannot happen), [2] links changed
    uint32_t *sc;             // entries handed out per shard (stride kRetStride)
    uint32_t per, cap, n;     // ids per shard, kRetShards * per, text positions (every link target is checked against n)
};
// `k` consecutive ids from shard `shard` (wave-wide: lane `leader` asks); ids past the
// shard's end are >= the returned limit and must not be used
PSA_DEV uint32_t ret_alloc(const RetList &R, uint32_t shard, uint32_t k, uint32_t leader, uint32_t *lim) {
    shard &= kRetShards - 1u;
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(R.sc + shard * kRetStride, k);
    base = (uint32_t)__shfl((int)base, (int)leader);
    *lim = shard * R.per + R.per;
    return shard * R.per + min(base, R.per);
}
// is id a handed-out entry?
PSA_DEV bool ret_used(const RetList &R, uint32_t id) {
    const uint32_t sh = id / R.per;
    return id - sh * R.per < min(__hip_atomic_load(R.sc + sh * kRetStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), R.per);
}
PSA_DEV uint64_t lnk_load(const unsigned long long *l, uint32_t id) {
    return __hip_atomic_load(l + id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
PSA_DEV void lnk_store(unsigned long long *l, uint32_t id, uint32_t T, uint32_t D) {
    __hip_atomic_store(l + id, (unsigned long long)D << 32 | T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the rank of suffix q whose stored rank r names a retired group (see above); links followed
// through exactly covering groups are stored back shortened
PSA_DEV uint32_t live_rank(const RetList &R, const uint32_t *rank, uint32_t q, uint32_t r) {
    uint32_t acc = 0, hops = 0;
    while (r & kRetired) {
        const uint32_t id = r & ~kRetired;
        const uint4 e = R.ent[id];
        const uint64_t l = lnk_load(R.lnk, id);
        uint32_t T = (uint32_t)l, D = (uint32_t)(l >> 32);
        if (q + D >= R.n) {
            atomicOr(R.cnt + 1, 1u);
            return 0;
        }
        uint32_t x = rank[q + D];
        bool shorter = false;
        while (x & kRetired) {  // the range is one retired group: its own link
            const uint32_t id2 = x & ~kRetired;
            const uint4 e2 = R.ent[id2];
            if (e2.x != T || e2.y != e.y) break;
            const uint64_t l2 = lnk_load(R.lnk, id2);
            if (q + D + (uint32_t)(l2 >> 32) >= R.n) break;
            T = (uint32_t)l2;
            D += (uint32_t)(l2 >> 32);
            x = rank[q + D];
            shorter = true;
            if (++hops > kMaxHops) break;
        }
        if (shorter) lnk_store(R.lnk, id, T, D);
        acc += e.x - T;
        q += D;
        r = x;
        if (++hops > kMaxHops) {
            atomicOr(R.cnt + 1, 1u);
            return 0;
        }
    }
    return acc + r;
}
// may group [g, g + size) with the one key K (>= 1) retire this step (the tag's step)?  Reads
// the target's size word while other waves may rewrite it: only an unrewritten word (the
// step's own tag) is taken; a target that retires or splits meanwhile is still a valid link
PSA_DEV bool retire_ok(const RetList &R, uint32_t g, uint32_t size, uint32_t K, uint32_t tag, const uint32_t *gsz) {
    if (!R.ent || K == 0 || K - 1 == g) return false;
    const uint32_t x = __hip_atomic_load(gsz + (K - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (x & kTag) == tag && (x & kSizeMask) == size;
}
PSA_DEV void retire_put(const RetList &R, uint32_t id, uint32_t g, uint32_t size, uint32_t q0, uint32_t K, uint32_t h) {
    R.ent[id] = make_uint4(g, size, q0, h);
    lnk_store(R.lnk, id, K - 1, h);
}
// pointer jumping over every entry's link (after the doubling): a link whose range one
// retired group covers exactly takes that group's link (read from src, written to dst);
// cnt[2] counts the links that changed
__global__ void __launch_bounds__(256) k_ret_jump(RetList R, const unsigned long long *src, unsigned long long *dst,
                                                  const uint32_t *rank) {
    uint32_t changed = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < R.cap; i += gridDim.x * blockDim.x) {
        if (!ret_used(R, i)) continue;
        const uint4 e = R.ent[i];
        const uint64_t l = src[i];
        uint32_t T = (uint32_t)l, D = (uint32_t)(l >> 32);
        const uint32_t x = e.z + D < R.n ? rank[e.z + D] : 0u;
        if (x & kRetired) {
            const uint4 e2 = R.ent[x & ~kRetired];
            if (e2.x == T && e2.y == e.y) {
                const uint64_t l2 = src[x & ~kRetired];
                T = (uint32_t)l2;
                D += (uint32_t)(l2 >> 32);
                ++changed;
            }
        }
        dst[i] = (unsigned long long)D << 32 | T;
    }
    if (__syncthreads_or(changed != 0) && threadIdx.x == 0) atomicAdd(R.cnt + 2, 1u);
}
// resolution (every live suffix's rank is its final slot): one wave per entry.  A: each
// member's final slot through its links into fin[slot] (members read from sa, nothing
// written that a rank read follows).  B: rank[q] = final slot, inv[final slot] = q.  C: the
// group's sa from inv.  (A final slot lies in the member's own group's range.)
template <int PH>
__global__ void __launch_bounds__(256) k_ret_resolve(RetList R, uint32_t *sa, uint32_t *rank, uint32_t *fin, uint32_t *inv) {
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < R.cap; i += waves) {
        if (!ret_used(R, i)) continue;
        const uint4 e = R.ent[i];
        for (uint32_t j = lane_id(); j < e.y; j += 64) {
            const uint32_t s = e.x + j;
            if (PH == 0) {
                const uint32_t q = sa[s];
                fin[s] = live_rank(R, rank, q, rank[q]);
            } else if (PH == 1) {
                const uint32_t q = sa[s], f = fin[s];
                if (f - e.x >= e.y) {  // (outside the group: cannot happen; the batch fails)
                    atomicOr(R.cnt + 1, 1u);
                    continue;
                }
                rank[q] = f;
                inv[f] = q;
            } else {
                sa[s] = inv[s];
            }
        }
    }
}

// per-step counters: suffixes sorted, slots still in groups after the step, largest group
// left.  Kept in kStatShards shards on lines of their own (one line per shard and counter
// set: a single address taking one atomic per wave serialises the whole launch), summed by
// k_stat_sum into the cnt words the host reads
constexpr uint32_t kStatShards = 64, kStatStride = 32;
struct StepStat {
    uint32_t *sh;  // [kStatShards][kStatStride]: sorted, active, maxsz
};
PSA_DEV void stat_put(const StepStat &ss, uint32_t slot, uint32_t sorted, uint32_t active, uint32_t mx) {
    uint32_t *c = ss.sh + (slot & (kStatShards - 1)) * kStatStride;
    if (sorted) atomicAdd(c, sorted);
    if (active) atomicAdd(c + 1, active);
    if (mx) atomicMax(c + 2, mx);
}
// (h_active / h_max: pinned host words also written, so the late doubling steps read their
// counts back without a copy each)
__global__ void k_stat_sum(const uint32_t *sh, uint32_t *sorted, uint32_t *active, uint32_t *maxsz,
                           uint32_t *h_active = nullptr, uint32_t *h_max = nullptr) {
    const uint32_t l = threadIdx.x;  // one wave
    uint32_t a = sh[l * kStatStride], b = sh[l * kStatStride + 1], c = sh[l * kStatStride + 2];
    for (int o = 32; o > 0; o >>= 1) {
        a += (uint32_t)__shfl_xor((int)a, o);
        b += (uint32_t)__shfl_xor((int)b, o);
        c = max(c, (uint32_t)__shfl_xor((int)c, o));
    }
    if (l == 0) {
        *sorted = a;
        *active = b;
        *maxsz = c;
        if (h_active) {  // (system scope: visible to the host once the step's event has passed)
            __hip_atomic_store(h_active, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(h_max, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

PSA_DEV uint32_t wave_incl_sum(uint32_t x) {
    const uint32_t lane = lane_id();
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x += y;
    }
    return x;
}
PSA_DEV uint32_t wave_sum(uint32_t x) {
    for (int o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o);
    return x;
}
PSA_DEV uint32_t wave_max(uint32_t x) {
    for (int o = 32; o > 0; o >>= 1) x = max(x, (uint32_t)__shfl_xor((int)x, o));
    return x;
}
// one stat_put per workgroup (every thread of the block calls it)
PSA_DEV void block_stat(const StepStat &ss, uint32_t sorted, uint32_t active, uint32_t mx) {
    __shared__ uint32_t red[3][4];
    sorted = wave_sum(sorted);
    active = wave_sum(active);
    mx = wave_max(mx);
    const uint32_t wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][wv] = sorted;
        red[1][wv] = active;
        red[2][wv] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t nw = blockDim.x >> 6;
        uint32_t a = 0, b = 0, c = 0;
        for (uint32_t w = 0; w < nw; ++w) {
            a += red[0][w];
            b += red[1][w];
            c = max(c, red[2][w]);
        }
        stat_put(ss, blockIdx.x, a, b, c);
    }
}
PSA_DEV uint64_t shfl64(uint64_t x, uint32_t src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, (int)src), hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), (int)src);
    return (uint64_t)hi << 32 | lo;
}
PSA_DEV uint64_t mask_le(uint32_t j) { return j >= 63 ? ~0ull : (2ull << j) - 1ull; }
PSA_DEV uint64_t mask_gt(uint32_t j) { return ~mask_le(j); }
PSA_DEV uint32_t hibit(uint64_t m) { return 63u - (uint32_t)__clzll((long long)m); }  // (m != 0)
PSA_DEV uint32_t lobit(uint64_t m) { return (uint32_t)__ffsll((long long)m) - 1u; }  // (m != 0)

// append long groups (wave-wide: every lane calls it; `valid` lanes hold one entry each)
PSA_DEV void push_long(const LongLists &L, bool valid, uint64_t ent) {
    const uint32_t cls = valid ? long_class((uint32_t)(ent >> 32)) : 255u;
    const uint32_t lane = lane_id();
    for (uint32_t c = 0; c < (uint32_t)kLongClasses; ++c) {
        const uint64_t m = __ballot(cls == c);
        if (!m) continue;
        const uint32_t leader = lobit(m);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&L.cnt[c], (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, (int)leader);
        if (cls == c) {
            const uint32_t at = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (at < L.cap[c]) L.lst[c][at] = ent;
            else atomicOr(&L.cnt[kLongClasses], 1u);  // (cannot happen: lists hold N / (class min) groups)
        }
    }
}

// The first groups, in one pass over the sorted keys (the group heads' max-scan by decoupled
// look-back over workgroups in the order they start).  A group starts at a key change and at
// every suffix shorter than `syms` symbols (its key holds its whole string, so its last symbol
// is 0: equal ones are equal strings, kept in position order by the stable sort and resolved as
// they are).  rank = group head index, sd = the doubling reach in suffix-array order (the
// sorted keys' kDlShift bits: steps whose key is a rank), act / gsz of the first groups (tag 0:
// step 0 sorts them).  A group's size is written at its start by its last element; every
// other slot writes its own gsz (0).  chain: one word per workgroup and the ticket after them,
// zeroed by the caller; a word is flag << 62 | (head + 1), the flag 1 for the workgroup's own
// last head (0: none in it), 2 for the last head at or before its end.
constexpr unsigned long long kG0Agg = 1ull << 62, kG0Incl = 2ull << 62, kG0Val = (1ull << 62) - 1ull;
PSA_DEV bool head_at(const uint64_t *skeys, uint32_t N, uint32_t r) {
    if (r == 0 || r >= N) return true;
    const uint64_t k = skeys[r] & kKeyMask;
    return k != (skeys[r - 1] & kKeyMask) || (k & 511u) == 0;
}
constexpr uint32_t kG0Rows = 16, kG0Slots = kG0Rows * 256;  // slots per workgroup: rows of 256
__global__ void __launch_bounds__(256) k_psa_groups0(uint32_t N, const uint32_t *sa, const uint64_t *skeys,
                                                     unsigned long long *chain, uint32_t *err, uint32_t *rank, uint16_t *sd,
                                                     uint8_t *act, uint32_t *gsz, StepStat ss) {
    __shared__ uint32_t s_bid, s_w[2][4], s_pre;
    const uint32_t nb = gridDim.x;
    if (threadIdx.x == 0) s_bid = atomicAdd((uint32_t *)(chain + nb), 1u);  // (tickets: look-back never waits on a later one)
    __syncthreads();
    const uint32_t bid = s_bid, base = bid * kG0Slots, lane = lane_id(), w = threadIdx.x >> 6;
    // every load first (rows of 256 slots; a slot's neighbours come from the next lanes, the
    // wave's edge lanes load theirs), so the block waits on memory once
    uint64_t kc[kG0Rows], ke[kG0Rows];
    uint32_t pp[kG0Rows];
#pragma unroll
    for (uint32_t i = 0; i < kG0Rows; ++i) {
        const uint32_t r = base + i * 256u + threadIdx.x;
        kc[i] = r < N ? skeys[r] : 0ull;
        ke[i] = lane == 0 ? (r > 0 && r <= N ? skeys[r - 1] : 0ull) : lane == 63 ? (r + 1 < N ? skeys[r + 1] : 0ull) : 0ull;
        pp[i] = r < N ? sa[r] : 0u;
    }
    // row i = slots base + 256 i + (0..255): inclusive max-scan of (head + 1) in slot order
    uint32_t hv[kG0Rows], hnm = 0, carry = 0;
#pragma unroll
    for (uint32_t i = 0; i < kG0Rows; ++i) {
        const uint32_t r = base + i * 256u + threadIdx.x;
        const uint64_t k = kc[i] & kKeyMask;
        // (every lane shuffles: a lane left out of a shuffle hands its neighbour nothing)
        const uint64_t sl = shfl64(kc[i], (lane + 63u) & 63u), sr = shfl64(kc[i], (lane + 1u) & 63u);
        const uint64_t kl = (lane == 0 ? ke[i] : sl) & kKeyMask;
        const uint64_t kr = (lane == 63 ? ke[i] : sr) & kKeyMask;
        const bool f = r < N && (r == 0 || k != kl || (k & 511u) == 0);
        if (r < N && (r + 1 >= N || kr != k || (kr & 511u) == 0)) hnm |= 1u << i;  // r + 1 starts the next group (or the end)
        uint32_t v = f ? r + 1u : 0u;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)v, o);
            if (lane >= o) v = max(v, y);
        }
        if (lane == 63) s_w[i & 1][w] = v;
        __syncthreads();  // (rows alternate between two exchange slots: one barrier per row)
        for (uint32_t x = 0; x < w; ++x) v = max(v, s_w[i & 1][x]);
        hv[i] = max(v, carry);
        carry = max(carry, max(max(s_w[i & 1][0], s_w[i & 1][1]), max(s_w[i & 1][2], s_w[i & 1][3])));
    }
    if (threadIdx.x == 0) {
        const uint32_t agg = carry;
        // a workgroup holding a head knows its inclusive value at once
        __hip_atomic_store(chain + bid, (agg || bid == 0 ? kG0Incl : kG0Agg) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t pre = 0, spins = 0;
        if (bid > 0 && !head_at(skeys, N, base)) {  // (its first slot's head lies before it)
            for (uint32_t j = bid - 1;;) {
                const unsigned long long x = __hip_atomic_load(chain + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!(x >> 62)) {
                    if (++spins > (1u << 24)) {  // (cannot happen: the batch fails loudly)
                        atomicOr(err, 1u);
                        break;
                    }
                    continue;
                }
                pre = max(pre, (uint32_t)(x & kG0Val));
                if ((x >> 62) == 2 || j == 0) break;
                --j;
            }
            if (!agg) __hip_atomic_store(chain + bid, kG0Incl | pre, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_pre = pre;
    }
    __syncthreads();
    const uint32_t pre = s_pre;
    uint32_t a_all = 0, mx = 0;
#pragma unroll
    for (uint32_t i = 0; i < kG0Rows; ++i) {
        const uint32_t r = base + i * 256u + threadIdx.x;
        if (r >= N) break;
        const bool hn = (hnm >> i) & 1u;
        const uint32_t hd = max(hv[i], pre) - 1u;
        rank[pp[i]] = hd;
        const uint32_t a = (hd != r || !hn) ? 1u : 0u;  // in a group of >= 2
        a_all += a;
        sd[r] = a ? (uint16_t)((kc[i] >> kDlShift) & 15u) : (uint16_t)0;
        act[r] = (uint8_t)a;
        if (!(hd == r && !hn)) gsz[r] = 0;  // (not the start of a group of >= 2)
        if (hn && hd != r) {                // the last element of a group of >= 2
            gsz[hd] = r - hd + 1;
            mx = max(mx, r - hd + 1);
        }
    }
    block_stat(ss, 0, a_all, mx);
}

// this step's keys: rank of the suffix h further on (+1), 0 past the doc end (step `it` of
// the doubling, h = syms << it: the suffix reaches h further inside its doc iff it < sd).
// Flat over the suffix array, 16 slots per thread: every scattered rank read of the step in
// flight at once
__global__ void __launch_bounds__(256) k_dbl_key(uint32_t N, uint32_t h, uint32_t it, const uint8_t *act, const uint32_t *sa,
                                                 const uint16_t *sd, const uint32_t *rank, uint32_t *key,
                                                 uint32_t *long_cnt, RetList R, uint32_t *err) {
    // (a rank read past the text -- a reach that overstates the doc, as corrupted sort keys
    // once gave -- is refused and fails the batch instead of faulting)
    const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (t0 < 8) long_cnt[t0] = 0;  // (the step's long-group lists start empty: k_dbl_win fills them)
    // (launched with one thread per piece: the loop runs once; see the step driver)
    for (uint32_t t = t0; (uint64_t)t * 16 < N; t += gridDim.x * blockDim.x) {
        const uint32_t s0 = t * 16;
        if (s0 + 16 <= N) {
            const uint4 av = *(const uint4 *)(act + s0);
            if ((av.x | av.y | av.z | av.w) == 0) continue;
            uint32_t p[16], k[16];
            uint16_t d[16];
            for (int q = 0; q < 4; ++q) *(uint4 *)(p + 4 * q) = *(const uint4 *)(sa + s0 + 4 * q);
            for (int q = 0; q < 2; ++q) *(uint4 *)(d + 8 * q) = *(const uint4 *)(sd + s0 + 8 * q);
            const uint32_t aw[4] = {av.x, av.y, av.z, av.w};
            bool any_ret = false, bad = false;
    #pragma unroll
            for (int i = 0; i < 16; ++i) {  // (slots outside groups get a key nobody reads)
                const bool want = ((aw[i >> 2] >> (8 * (i & 3))) & 0xffu) && it < d[i];
                const uint32_t q = p[i] + h;
                k[i] = want && q < N ? rank[q] + 1u : 0u;
                bad = bad || (want && q >= N);
                any_ret = any_ret || (k[i] != 0 && ((k[i] - 1u) & kRetired) != 0);
            }
            if (bad) atomicOr(err, 2u);
            if (any_ret) {  // (ranks of retired groups: through their links)
    #pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (k[i] != 0 && ((k[i] - 1u) & kRetired)) k[i] = live_rank(R, rank, p[i] + h, k[i] - 1u) + 1u;
            }
            for (int q = 0; q < 4; ++q) *(uint4 *)(key + s0 + 4 * q) = *(const uint4 *)(k + 4 * q);
        } else {
            for (uint32_t s = s0; s < N; ++s)
                if (act[s]) {
                    uint32_t r = 0;
                    if (it < sd[s] && sa[s] + h >= N) {
                        atomicOr(err, 2u);
                    } else if (it < sd[s]) {
                        r = rank[sa[s] + h];
                        if (r & kRetired) r = live_rank(R, rank, sa[s] + h, r);
                        ++r;
                    }
                    key[s] = r;
                }
        }
    }
}

// One wave per 64-slot window: the groups of <= 64 that start in it (and so end within
// the next window) are sorted where they lie, 128 slots over 64 lanes (A: slot b + lane,
// B: slot b + 64 + lane); a longer group starting in it goes to its class list.  Each
// member ranks itself against its group's keys (staged in LDS): its sorted position
// (key, then index -- stable), the members before it with an equal key (0: it heads a
// subgroup) and the members with its key (the subgroup size).  So it writes its own
// destination, its new rank (only where it changes) and act / gsz of the next step's
// groups without any sorting network.
struct WinElem {
    bool mem;
    uint32_t c, z, i, key, p, d;  // group start lane, size, index in the group, key, payload
};
PSA_DEV void win_rank(const WinElem &e, const uint32_t *lk, uint32_t smax, uint32_t &lt, uint32_t &eqb, uint32_t &eqt) {
    lt = eqb = eqt = 0;
    for (uint32_t t = 0; t < smax; ++t) {  // (smax is wave-uniform)
        const uint32_t kt = lk[(e.c + t) & 127u];
        if (e.mem && t < e.z && t != e.i) {
            lt += (kt < e.key || (kt == e.key && t < e.i)) ? 1u : 0u;
            eqb += (kt == e.key && t < e.i) ? 1u : 0u;
            eqt += kt == e.key ? 1u : 0u;
        }
    }
}
PSA_DEV void win_put(const WinElem &e, uint32_t b, uint32_t lt, uint32_t eqb, uint32_t eqt, uint32_t tag, uint32_t *sa,
                     uint16_t *sd, uint8_t *act, uint32_t *gsz, uint32_t *rank, uint32_t &ac, uint32_t &mx) {
    const uint32_t dst = b + e.c + lt;
    // key 0: a complete suffix, a subgroup of its own (equal complete strings stay in index order)
    const bool head = e.key == 0 || eqb == 0;
    const uint32_t hd = e.key == 0 ? lt : lt - eqb, size = e.key == 0 ? 1u : eqt + 1u;
    const bool grp = e.key != 0 && size >= 2;
    sa[dst] = e.p;
    sd[dst] = (uint16_t)e.d;
    act[dst] = grp ? 1 : 0;
    gsz[dst] = head && grp ? (size | (tag ^ kTag)) : 0u;
    if (hd != 0) rank[e.p] = b + e.c + hd;
    ac += grp;
    if (head && grp) mx = max(mx, size);
}
__global__ void __launch_bounds__(256) k_dbl_win(uint32_t N, uint32_t tag, uint32_t h, uint32_t *sa, uint16_t *sd, uint8_t *act,
                                                 uint32_t *gsz, const uint32_t *key, uint32_t *rank, LongLists L,
                                                 StepStat ss, RetList R, uint32_t split) {
    __shared__ uint32_t lks[4][128];
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    uint32_t *lk = lks[wv];
    const uint32_t nwin = (N + 63) / 64;
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    uint32_t sorted = 0, active = 0, mx = 0;
    uint64_t pend = 0;  // pending long groups, lane i holds entry i
    uint32_t npend = 0;
    // a wave takes 64 windows at a time and visits only those holding an unsorted slot
    // (one 64-byte act load per lane finds them: late steps leave most windows empty, and
    // testing them one by one was a dependent load per window)
    // (lane l of chunk c tests window l * nch + c: a run of busy windows -- a template's
    // copies -- is dealt over many waves instead of queueing on one)
    // (split > 1, small rounds: `split` waves share a chunk, each taking every split-th of its
    // busy windows -- a single-instance round of 12 M positions has ~2,900 chunks, under 3 waves
    // per SIMD for a kernel that waits on scattered loads)
    const uint32_t nch = (nwin + 63) / 64;
    const uint32_t units = nch * split;
    for (uint32_t un = blockIdx.x * (blockDim.x >> 6) + wv; un < units; un += waves) {
      const uint32_t c = un / split, sub = un - c * split;
      uint64_t todo;
      {
        const uint32_t wl = lane * nch + c, s0 = wl * 64;
        bool any = false;
        if (wl < nwin) {
            if (s0 + 64 <= N) {
                const uint4 *a4 = (const uint4 *)(act + s0);
                const uint4 x = a4[0], y = a4[1], z = a4[2], u = a4[3];
                any = ((x.x | x.y | x.z | x.w) | (y.x | y.y | y.z | y.w) | (z.x | z.y | z.z | z.w) |
                       (u.x | u.y | u.z | u.w)) != 0;
            } else {
                for (uint32_t q = s0; q < N; ++q) any |= act[q] != 0;
            }
        }
        // (a shared chunk: this wave's windows are its lanes l with l % split == sub -- a fixed
        // owner per window.  Dealing the busy windows by their rank instead hangs: act changes
        // while the chunk's waves run, so their busy masks, and ranks, differ)
        todo = __ballot(any && lane % split == sub);
      }
      while (todo) {
        const uint32_t w = lobit(todo) * nch + c;
        todo &= todo - 1;
        const uint32_t b = w * 64, sA = b + lane, sB = b + 64 + lane;
        const bool inA = sA < N;
        const uint32_t g = inA ? gsz[sA] : 0u;
        const bool start = (g & kTag) == tag && (g & kSizeMask) >= 2;
        const uint32_t gs = g & kSizeMask;
        const uint64_t S = __ballot(start && gs <= kWinMax);
        const uint64_t Lg = __ballot(start && gs > kWinMax);
        if (Lg) {  // (at most one: it runs past the window)
            const uint32_t l = lobit(Lg);
            const uint32_t sz = (uint32_t)__shfl((int)gs, (int)l);
            if (lane == npend) pend = (uint64_t)(b + l) | (uint64_t)sz << 32;
            if (++npend == 64) {
                push_long(L, true, pend);
                npend = 0;
            }
        }
        if (!S) continue;
        // membership: the last small start at or before the slot, if the slot lies inside it
        const uint32_t cA = (S & mask_le(lane)) ? hibit(S & mask_le(lane)) : 64u;
        const uint32_t cB = hibit(S);
        const uint32_t zA = (uint32_t)__shfl((int)gs, (int)(cA & 63u)), zB = (uint32_t)__shfl((int)gs, (int)cB);
        WinElem A{cA < 64 && lane < cA + zA, cA & 63u, zA, lane - cA, 0, 0, 0};
        WinElem B{64 + lane < cB + zB, cB, zB, 64 + lane - cB, 0, 0, 0};
        if (A.mem) A.key = key[sA];
        if (B.mem) B.key = key[sB];
        {
            // every group keeps one key (a repeat longer than 2h): the groups stay as they are,
            // only their sizes move to the next step's tag
            const uint32_t k0A = (uint32_t)__shfl((int)A.key, (int)A.c), k0B = (uint32_t)__shfl((int)A.key, (int)cB);
            const uint64_t split = __ballot(A.mem && (A.key != k0A || A.key == 0)) |
                                   __ballot(B.mem && (B.key != k0B || B.key == 0));
            if (!split) {
                // groups that are shifted copies of another leave the doubling (see RetList)
                uint64_t Rm = __ballot(((S >> lane) & 1ull) && retire_ok(R, b + lane, gs, A.key, tag, gsz));
                uint32_t id = 0;
                if (Rm) {
                    uint32_t lim;
                    const uint32_t base = ret_alloc(R, w, (uint32_t)__popcll(Rm), 0, &lim);
                    id = base + (uint32_t)__popcll(Rm & ((1ull << lane) - 1ull));
                    Rm &= __ballot(id < lim);  // (past the shard's end: those groups stay; every id below it is written)
                }
                const bool rA = A.mem && ((Rm >> A.c) & 1ull), rB = B.mem && ((Rm >> B.c) & 1ull);
                const uint32_t idA = (uint32_t)__shfl((int)id, (int)A.c), idB = (uint32_t)__shfl((int)id, (int)B.c);
                uint32_t pA = 0;
                if (rA) {
                    act[sA] = 0;
                    pA = sa[sA];
                    rank[pA] = idA | kRetired;
                }
                if (rB) {
                    act[sB] = 0;
                    rank[sa[sB]] = idB | kRetired;
                }
                if ((S >> lane) & 1ull) {
                    if ((Rm >> lane) & 1ull) {
                        gsz[sA] = 0;
                        retire_put(R, id, b + lane, gs, pA, A.key, h);
                    } else {
                        gsz[sA] = gs | (tag ^ kTag);
                        mx = max(mx, gs);
                    }
                }
                const uint32_t m = (uint32_t)__popcll(__ballot(A.mem)) + (uint32_t)__popcll(__ballot(B.mem));
                const uint32_t mr = (uint32_t)__popcll(__ballot(rA)) + (uint32_t)__popcll(__ballot(rB));
                sorted += m;
                active += lane == 0 ? m - mr : 0u;
                continue;
            }
        }
        if (A.mem) {
            A.p = sa[sA];
            A.d = sd[sA];
        }
        if (B.mem) {
            B.p = sa[sB];
            B.d = sd[sB];
        }
        lk[lane] = A.key;
        lk[64 + lane] = B.key;
        const uint32_t smax = wave_max((S >> lane) & 1ull ? gs : 0u);
        uint32_t lA, eA, tA, lB, eB, tB;
        win_rank(A, lk, smax, lA, eA, tA);
        win_rank(B, lk, smax, lB, eB, tB);
        uint32_t ac = 0;
        if (A.mem) win_put(A, b, lA, eA, tA, tag, sa, sd, act, gsz, rank, ac, mx);
        if (B.mem) win_put(B, b, lB, eB, tB, tag, sa, sd, act, gsz, rank, ac, mx);
        sorted += (uint32_t)__popcll(__ballot(A.mem)) + (uint32_t)__popcll(__ballot(B.mem));
        active += ac;
      }
    }
    push_long(L, lane < npend, pend);
    active = wave_sum(active);
    mx = wave_max(mx);
    if (lane == 0) stat_put(ss, blockIdx.x * 4 + wv, sorted, active, mx);
}

// The subgroups of one sorted group (positions q = 0..size-1 in sorted order, any layout):
// writes element q's slot and reports whether it opens / continues a group.  Shared by the
// register and LDS sorters through a per-position view.
PSA_DEV void put_sorted(uint32_t start, uint32_t q, uint32_t p, uint32_t d, uint32_t key, bool head, uint32_t hd,
                        uint32_t nxt, uint32_t tag, uint32_t *sa, uint16_t *sd, uint8_t *act, uint32_t *gsz, uint32_t *rank,
                        uint32_t &ac, uint32_t &mx) {
    const uint32_t dst = start + q, szn = nxt - q;
#ifdef PX_PSA_DEBUG
    if (szn > 0x10000000u) printf("put_sorted: start %u q %u nxt %u head %d hd %u key %u\n", start, q, nxt, (int)head, hd, key);
#endif
    sa[dst] = p;
    sd[dst] = (uint16_t)d;
    const bool grp = key != 0 && !(head && szn == 1);
    act[dst] = grp ? 1 : 0;
    gsz[dst] = head && grp ? (szn | (tag ^ kTag)) : 0u;
    if (hd != 0) rank[p] = start + hd;
    ac += grp;
    if (head && grp) mx = max(mx, szn);
}

// One wave per group of 65..64*E suffixes: E elements per lane (lane l holds positions
// l*E .. l*E+E-1), bitonic sort in registers; payloads through LDS.
template <uint32_t E>
__global__ void __launch_bounds__(256) k_dbl_reg(const uint64_t *list, const uint32_t *cnt_p, uint32_t tag, uint32_t h,
                                                 uint32_t *sa, uint16_t *sd, uint8_t *act, uint32_t *gsz, const uint32_t *key,
                                                 uint32_t *rank, StepStat ss, RetList R) {
    __shared__ uint32_t lp[4][64 * E];
    __shared__ uint16_t ld[4][64 * E];
    const uint32_t cnt = __hip_atomic_load(cnt_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    uint32_t sorted = 0, active = 0, mx = 0;
    for (uint32_t gi = blockIdx.x * (blockDim.x >> 6) + wv; gi < cnt; gi += waves) {
        const uint64_t ent = list[gi];
        const uint32_t start = (uint32_t)ent, size = (uint32_t)(ent >> 32);
        uint64_t x[E];
        const uint32_t key0 = key[start];
        bool split = false;
#pragma unroll
        for (uint32_t r = 0; r < E; ++r) {
            const uint32_t i = lane * E + r;
            const uint32_t k = i < size ? key[start + i] : key0;
            x[r] = i < size ? (uint64_t)k << 11 | i : ~0ull;
            split = split || k != key0 || k == 0;
        }
        if (!__ballot(split)) {  // one key: the group stays as it is (see k_dbl_win) or retires
            uint32_t id = kNoPos;
            if (retire_ok(R, start, size, key0, tag, gsz)) {
                uint32_t lim;
                id = ret_alloc(R, gi, 1, 0, &lim);
                if (id >= lim) id = kNoPos;
            }
            sorted += size;
            if (id != kNoPos) {
                uint32_t p0 = 0;
#pragma unroll
                for (uint32_t r = 0; r < E; ++r) {
                    const uint32_t i = lane * E + r;
                    if (i < size) {
                        act[start + i] = 0;
                        const uint32_t p = sa[start + i];
                        rank[p] = id | kRetired;
                        if (i == 0) p0 = p;
                    }
                }
                if (lane == 0) {
                    gsz[start] = 0;
                    retire_put(R, id, start, size, p0, key0, h);
                }
                continue;
            }
            if (lane == 0) gsz[start] = size | (tag ^ kTag);
            mx = max(mx, size);
            active += size;
            continue;
        }
#pragma unroll
        for (uint32_t r = 0; r < E; ++r) {
            const uint32_t i = lane * E + r;
            if (i < size) {
                lp[wv][i] = sa[start + i];
                ld[wv][i] = sd[start + i];
            }
        }
#pragma unroll
        for (uint32_t k = 2; k <= 64 * E; k <<= 1)
#pragma unroll
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                if (j < E) {
#pragma unroll
                    for (uint32_t r = 0; r < E; ++r) {
                        if (r & j) continue;
                        const uint32_t i = lane * E + r;
                        const bool up = (i & k) == 0;
                        const uint64_t a = x[r], c = x[r | j];
                        if (up ? a > c : a < c) {
                            x[r] = c;
                            x[r | j] = a;
                        }
                    }
                } else {
                    const uint32_t lj = j / E;
                    const bool lower = (lane & lj) == 0;
#pragma unroll
                    for (uint32_t r = 0; r < E; ++r) {
                        const uint64_t o = shfl64(x[r], lane ^ lj);
                        const bool up = ((lane * E + r) & k) == 0;
                        x[r] = up == lower ? (o < x[r] ? o : x[r]) : (o > x[r] ? o : x[r]);
                    }
                }
            }
        // subgroup heads as a lane mask over the lane's E positions; the head at or before a
        // position and the next one after it come from the mask and two cross-lane scans
        const uint32_t prevk = (uint32_t)__shfl_up((int)(uint32_t)(x[E - 1] >> 11), 1);
        uint32_t hm = 0;
#pragma unroll
        for (uint32_t r = 0; r < E; ++r) {
            const uint32_t i = lane * E + r;
            const uint32_t kr = (uint32_t)(x[r] >> 11), pk = r ? (uint32_t)(x[r - 1] >> 11) : prevk;
            if (i < size && (i == 0 || kr != pk || kr == 0)) hm |= 1u << r;
        }
        uint32_t lmax = hm ? lane * E + (31u - (uint32_t)__clz(hm)) + 1u : 0u;  // last head + 1 (0: none)
        uint32_t lmin = hm ? lane * E + (uint32_t)__ffs(hm) - 1u : 0xffffffffu;  // first head
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)lmax, o), z = (uint32_t)__shfl_down((int)lmin, o);
            if (lane >= o) lmax = max(lmax, y);
            if (lane + o < 64) lmin = min(lmin, z);
        }
        // (shuffles outside the selects: a lane that reads an inactive lane gets 0)
        const uint32_t up1 = (uint32_t)__shfl_up((int)lmax, 1), dn1 = (uint32_t)__shfl_down((int)lmin, 1);
        const uint32_t before = lane ? up1 - 1u : 0u;         // head before the lane
        const uint32_t after = lane < 63 ? dn1 : 0xffffffffu;  // head after it
        uint32_t ac = 0;
#pragma unroll
        for (uint32_t r = 0; r < E; ++r) {
            const uint32_t i = lane * E + r;
            if (i >= size) continue;
            const uint32_t le = hm & ((2u << r) - 1u), gt = hm & ~((2u << r) - 1u);
            const uint32_t hd = le ? lane * E + (31u - (uint32_t)__clz(le)) : before;
            const uint32_t nx = min(gt ? lane * E + (uint32_t)__ffs(gt) - 1u : after, size);
            const uint32_t o = (uint32_t)(x[r] & 2047u);
            put_sorted(start, i, lp[wv][o], ld[wv][o], (uint32_t)(x[r] >> 11), (hm >> r) & 1u, hd, nx, tag, sa, sd, act,
                       gsz, rank, ac, mx);
        }
        sorted += size;
        active += wave_sum(ac);
    }
    mx = wave_max(mx);
    if (lane == 0) stat_put(ss, blockIdx.x * 4 + wv, sorted, active, mx);
}

// bitonic network over sk[0 .. P) in LDS (256 threads; PMAX >= P, both powers of two >= 512):
// stage (kk, j) compares pair q's elements i = q with a 0 bit inserted at j, and i | j
// A stage with j <= 32 stays inside each wave's own elements (wave w takes pairs 64 w .. 64 w + 63
// of every 256, i.e. elements 128 w .. 128 w + 127 of every 512), so it needs no workgroup barrier:
// only the stages with j >= 64 and the last stage of each kk (the next kk starts at j = kk / 2)
// wait for the other waves.  (LDS operations of one wave complete in order; the wave barrier keeps
// the compiler from moving them across stages.)
template <uint32_t P>
PSA_DEV void blk_bitonic(uint64_t *sk) {
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (uint32_t kk = 2; kk <= P; kk <<= 1) {
#pragma unroll
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (uint32_t m = 0; m < P / 512; ++m) {
                const uint32_t q = tid + m * 256;
                const uint32_t i = ((q & ~(j - 1u)) << 1) | (q & (j - 1u)), l = i | j;
                const bool up = (i & kk) == 0;
                const uint64_t x = sk[i], y = sk[l];
                if (up ? x > y : x < y) {
                    sk[i] = y;
                    sk[l] = x;
                }
            }
            if (j >= 64 || j == 1) {
                __syncthreads();
            } else {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    }
}
// any power-of-two P (256 .. kMedMax): the runtime-sized network
PSA_DEV void blk_bitonic_any(uint64_t *sk, uint32_t P) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t kk = 2; kk <= P; kk <<= 1)
        for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
            for (uint32_t i = tid; i < P; i += 256) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const bool up = (i & kk) == 0;
                    const uint64_t x = sk[i], y = sk[l];
                    if (up ? x > y : x < y) {
                        sk[i] = y;
                        sk[l] = x;
                    }
                }
            }
            __syncthreads();
        }
}

// one workgroup per group of kRegMax+1 .. kMedMax: bitonic sort of the keys in LDS; then
// each thread takes C = P / 256 consecutive positions: their heads as a mask, their payloads
// gathered before any slot of the group is rewritten, and the subgroup bounds across threads
// from two block scans
__global__ void __launch_bounds__(256) k_dbl_blk(const uint64_t *list, const uint32_t *cnt_p, uint32_t tag, uint32_t h,
                                                 uint32_t *sa, uint16_t *sd, uint8_t *act, uint32_t *gsz, const uint32_t *key,
                                                 uint32_t *rank, StepStat ss, RetList R) {
    __shared__ uint64_t sk[kMedMax];
    __shared__ uint32_t sl[256], sf[256];
    constexpr uint32_t kC = kMedMax / 256;
    const uint32_t cnt = __hip_atomic_load(cnt_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t tid = threadIdx.x;
    uint32_t sorted = 0, active = 0, mx = 0;
    for (uint32_t gi = blockIdx.x; gi < cnt; gi += gridDim.x) {
        const uint64_t ent = list[gi];
        const uint32_t start = (uint32_t)ent, size = (uint32_t)(ent >> 32);
        uint32_t P = 256;
        while (P < size) P <<= 1;
        const uint32_t key0 = key[start];
        bool split = false;
        for (uint32_t i = tid; i < P; i += 256) {
            const uint32_t k = i < size ? key[start + i] : key0;
            split = split || k != key0 || k == 0;
            sk[i] = i < size ? (uint64_t)k << 12 | i : ~0ull;
        }
        if (!__syncthreads_or(split)) {  // one key: the group stays as it is (see k_dbl_win) or retires
            __shared__ uint32_t s_id;
            if (tid == 0) {
                uint32_t id = kNoPos;
                if (retire_ok(R, start, size, key0, tag, gsz)) {
                    const uint32_t sh = gi & (kRetShards - 1u);
                    id = atomicAdd(R.sc + sh * kRetStride, 1u);
                    id = id < R.per ? sh * R.per + id : kNoPos;
                }
                s_id = id;
            }
            __syncthreads();
            const uint32_t id = s_id;
            sorted += size;
            if (id != kNoPos) {
                uint32_t p0 = 0;
                for (uint32_t i = tid; i < size; i += 256) {
                    act[start + i] = 0;
                    const uint32_t p = sa[start + i];
                    rank[p] = id | kRetired;
                    if (i == 0) p0 = p;
                }
                if (tid == 0) {
                    gsz[start] = 0;
                    retire_put(R, id, start, size, p0, key0, h);
                }
            } else {
                if (tid == 0) {
                    gsz[start] = size | (tag ^ kTag);
                    active += size;
                }
                mx = max(mx, size);
            }
            __syncthreads();  // (s_id is rewritten by the next group)
            continue;  // (the barrier above: nobody reads sk any more)
        }
        // (the network at compile-time sizes: every thread takes P / 512 pairs per stage; the
        // runtime-sized loops spent more scalar than vector instructions, profiles/r05ze_sq_summary.txt)
        if (P == 1024) blk_bitonic<1024>(sk);
        else if (P == 2048) blk_bitonic<2048>(sk);
        else if (P == 4096) blk_bitonic<4096>(sk);
        else blk_bitonic_any(sk, P);
        const uint32_t C = P / 256, i0 = tid * C;
        uint32_t hm = 0, pv[kC], dv[kC];
#pragma unroll
        for (uint32_t c = 0; c < kC; ++c) {
            const uint32_t i = i0 + c;
            if (c < C && i < size) {
                const uint64_t x = sk[i];
                const uint32_t k = (uint32_t)(x >> 12);
                if (i == 0 || k != (uint32_t)(sk[i - 1] >> 12) || k == 0) hm |= 1u << c;
                const uint32_t o = (uint32_t)(x & 4095u);
                pv[c] = sa[start + o];
                dv[c] = sd[start + o];
            }
        }
        sl[tid] = hm ? i0 + (31u - (uint32_t)__clz(hm)) + 1u : 0u;
        sf[tid] = hm ? i0 + (uint32_t)__ffs(hm) - 1u : 0xffffffffu;
        __syncthreads();  // (every payload of the group is read: its slots may be rewritten)
        for (uint32_t o = 1; o < 256; o <<= 1) {
            const uint32_t a = tid >= o ? max(sl[tid], sl[tid - o]) : sl[tid];
            const uint32_t b = tid + o < 256 ? min(sf[tid], sf[tid + o]) : sf[tid];
            __syncthreads();
            sl[tid] = a;
            sf[tid] = b;
            __syncthreads();
        }
        const uint32_t before = tid ? sl[tid - 1] - 1u : 0u, after = tid < 255 ? sf[tid + 1] : 0xffffffffu;
        uint32_t ac = 0;
#pragma unroll
        for (uint32_t c = 0; c < kC; ++c) {
            const uint32_t i = i0 + c;
            if (c < C && i < size) {
                const uint32_t le = hm & ((2u << c) - 1u), gt = hm & ~((2u << c) - 1u);
                const uint32_t hd = le ? i0 + (31u - (uint32_t)__clz(le)) : before;
                const uint32_t nx = min(gt ? i0 + (uint32_t)__ffs(gt) - 1u : after, size);
                put_sorted(start, i, pv[c], dv[c], (uint32_t)(sk[i] >> 12), (hm >> c) & 1u, hd, nx, tag, sa, sd, act, gsz,
                           rank, ac, mx);
            }
        }
        active += ac;
        sorted += size;
        __syncthreads();  // (sk is refilled by the next group)
    }
    block_stat(ss, tid == 0 ? sorted : 0u, active, mx);
}

// big groups (host-driven steps): gather every member with key (group << 32 | key), sort
// each group by its key (px_sort.hip: stable, ties keep suffix-array order), place back,
// heads by a max-scan, then ranks and subgroups.  boff = exclusive prefix of the groups'
// sizes (host-computed).  PACKED (fewer than 65,536 groups): the member's distance rides in
// the key's top 16 bits and its position is the sorted value, so placing a member back
// reads nothing scattered (otherwise the value is the gather index and the position and
// distance come from gp / gd).
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
// flat over the T gathered members: a block's 256 members span at most two groups (every
// big group has > 4,096 members), found by one search of boff per block
template <bool PACKED>
// Keys are made relative to the group's shard (rank + 1 - the shard's first slot, 0 kept for a
// complete suffix): the rank h further on lies in the same shard, so the sort needs the bit
// length of the largest shard (23-24 bits, 3 passes of 8) instead of 32 (4 passes).
__global__ void __launch_bounds__(256) k_big_gather(uint32_t T, uint32_t nb, const uint64_t *list, const uint32_t *boff,
                                                    const uint32_t *sa, const uint16_t *sd, const uint32_t *key,
                                                    uint64_t *ck, uint32_t *cv, uint32_t *gp, uint16_t *gd, StepStat ss,
                                                    const PsaShard *shards, uint32_t nshards) {
    __shared__ uint32_t sb, sbase[2];
    const uint32_t k0 = blockIdx.x * blockDim.x, k = k0 + threadIdx.x;
    if (threadIdx.x == 0) {  // the group holding k0: last b with boff[b] <= k0
        uint32_t lo = 0, hi = nb;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (boff[mid] <= k0) lo = mid;
            else hi = mid;
        }
        sb = lo;
        // the shard bases of the (at most two) groups the block's members are in
        sbase[0] = shards[shard_of_rank(shards, nshards, (uint32_t)list[lo])].base;
        sbase[1] = lo + 1 < nb ? shards[shard_of_rank(shards, nshards, (uint32_t)list[lo + 1])].base : 0u;
    }
    __syncthreads();
    if (k >= T) return;
    uint32_t b = sb, sbi = 0;
    if (b + 1 < nb && boff[b + 1] <= k) ++b, sbi = 1;
    const uint64_t ent = list[b];
    const uint32_t start = (uint32_t)ent, o = boff[b], i = k - o;
    const uint32_t kr = key[start + i], rel = kr ? kr - sbase[sbi] : 0u;
    if (PACKED) {
        ck[k] = (uint64_t)sd[start + i] << 48 | (uint64_t)b << 32 | rel;
        cv[k] = sa[start + i];
    } else {
        ck[k] = (uint64_t)b << 32 | rel;
        cv[k] = k;
        gp[k] = sa[start + i];
        gd[k] = sd[start + i];
    }
    if (i == 0) stat_put(ss, b, (uint32_t)(ent >> 32), 0, 0);
}
// the segments of the sorts (px_sort.hip): the round's shards, the big groups
__global__ void __launch_bounds__(256) k_psa_segs(uint32_t ns, const PsaShard *sh, uint32_t *start, uint32_t *len) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < ns) {
        start[i] = sh[i].base;
        len[i] = sh[i].len;
    }
}
__global__ void __launch_bounds__(256) k_big_segs(uint32_t nb, const uint64_t *list, uint32_t *len) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nb) len[i] = (uint32_t)(list[i] >> 32);
}
// The big groups placed back in one pass (what k_big_head, k_big_next, their two scans and
// k_big_put did): a subgroup starts at a group's first member, at a key change and at every key
// 0; the head at or before each member comes from a max-scan by decoupled look-back over
// workgroups of kG0Slots members (k_psa_groups0's scheme); a subgroup's size is written at its
// head by its last member.  chain: one word per workgroup and the ticket, zeroed by the caller.
template <bool PACKED>
__global__ void __launch_bounds__(256) k_big_place(uint32_t T, const uint64_t *list, const uint32_t *boff, const uint64_t *ck2,
                                                   const uint32_t *cv2, const uint32_t *gp, const uint16_t *gd, uint32_t tag,
                                                   unsigned long long *chain, uint32_t *err, uint32_t *sa, uint16_t *sd,
                                                   uint8_t *act, uint32_t *gsz, uint32_t *rank, StepStat ss) {
    __shared__ uint32_t s_bid, s_w[2][4], s_pre;
    const uint32_t nb = gridDim.x;
    if (threadIdx.x == 0) s_bid = atomicAdd((uint32_t *)(chain + nb), 1u);
    __syncthreads();
    const uint32_t bid = s_bid, base = bid * kG0Slots, lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t gmask = PACKED ? 0xffffu : 0xffffffffu;
    uint64_t kc[kG0Rows], ke[kG0Rows];
    uint32_t vv[kG0Rows];
#pragma unroll
    for (uint32_t i = 0; i < kG0Rows; ++i) {
        const uint32_t k = base + i * 256u + threadIdx.x;
        kc[i] = k < T ? ck2[k] : 0ull;
        ke[i] = lane == 0 ? (k > 0 && k <= T ? ck2[k - 1] : 0ull) : lane == 63 ? (k + 1 < T ? ck2[k + 1] : 0ull) : 0ull;
        vv[i] = k < T ? cv2[k] : 0u;
    }
    // (a member's group is (c >> 32) & gmask, its key the low word)
    auto head_of = [&](uint64_t c, uint64_t cl, uint32_t k) {
        return k == 0 || (((c >> 32) ^ (cl >> 32)) & gmask) != 0 || (uint32_t)c != (uint32_t)cl || (uint32_t)c == 0;
    };
    uint32_t hv[kG0Rows], hnm = 0, carry = 0;
#pragma unroll
    for (uint32_t i = 0; i < kG0Rows; ++i) {
        const uint32_t k = base + i * 256u + threadIdx.x;
        const uint64_t sl = shfl64(kc[i], (lane + 63u) & 63u), sr = shfl64(kc[i], (lane + 1u) & 63u);
        const uint64_t cl = lane == 0 ? ke[i] : sl, cr = lane == 63 ? ke[i] : sr;
        const bool f = k < T && head_of(kc[i], cl, k);
        if (k < T && (k + 1 >= T || head_of(cr, kc[i], k + 1))) hnm |= 1u << i;
        uint32_t v = f ? k + 1u : 0u;
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)v, o);
            if (lane >= o) v = max(v, y);
        }
        if (lane == 63) s_w[i & 1][w] = v;
        __syncthreads();
        for (uint32_t x = 0; x < w; ++x) v = max(v, s_w[i & 1][x]);
        hv[i] = max(v, carry);
        carry = max(carry, max(max(s_w[i & 1][0], s_w[i & 1][1]), max(s_w[i & 1][2], s_w[i & 1][3])));
    }
    if (threadIdx.x == 0) {
        const uint32_t agg = carry;
        __hip_atomic_store(chain + bid, (agg || bid == 0 ? kG0Incl : kG0Agg) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t pre = 0, spins = 0;
        const bool first_head = base == 0 || head_of(ck2[base], ck2[base - 1], base);
        if (bid > 0 && !first_head) {
            for (uint32_t j = bid - 1;;) {
                const unsigned long long x = __hip_atomic_load(chain + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!(x >> 62)) {
                    if (++spins > (1u << 24)) {
                        atomicOr(err, 1u);
                        break;
                    }
                    continue;
                }
                pre = max(pre, (uint32_t)(x & kG0Val));
                if ((x >> 62) == 2 || j == 0) break;
                --j;
            }
            if (!agg) __hip_atomic_store(chain + bid, kG0Incl | pre, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_pre = pre;
    }
    __syncthreads();
    const uint32_t pre = s_pre;
    uint32_t ac = 0, mx = 0;
#pragma unroll
    for (uint32_t i = 0; i < kG0Rows; ++i) {
        const uint32_t k = base + i * 256u + threadIdx.x;
        if (k >= T) break;
        const uint64_t c = kc[i];
        const uint32_t b = (uint32_t)(c >> 32) & gmask, key = (uint32_t)c, o = boff[b], start = (uint32_t)list[b];
        const uint32_t hg = max(hv[i], pre) - 1u;  // the head at or before k (T coordinates)
        const bool f = hg == k, hn = (hnm >> i) & 1u;
        const uint32_t v = vv[i], p = PACKED ? v : gp[v], d = PACKED ? (uint32_t)(c >> 48) : gd[v];
        const uint32_t q = k - o, dst = start + q, hd = hg - o;
        sa[dst] = p;
        sd[dst] = (uint16_t)d;
        const bool grp = key != 0 && !(f && hn);  // (a head followed by a head: a subgroup of one)
        act[dst] = grp ? 1 : 0;
        if (!(f && grp)) gsz[dst] = 0;  // (a subgroup's size is written at its head by its last member)
        if (hd != 0) rank[p] = start + hd;
        ac += grp;
        if (hn && grp) {  // the last member of a subgroup of >= 2
            const uint32_t size = k - hg + 1u;
            gsz[start + hd] = size | (tag ^ kTag);
            mx = max(mx, size);
        }
    }
    block_stat(ss, 0, ac, mx);
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

// Block-level ANSV: one workgroup per kAnsvBlock ranks.  Each wave first resolves its
// 64-rank sub-blocks by binary lifting; an element with no smaller value on a side
// inside its sub-block then looks for the nearest sub-block of the workgroup whose minimum is
// smaller (one ballot over the 64 sub-block minima in LDS) and, inside it, for the nearest
// smaller element (one ballot over its 64 values in LDS).  Each wave computes the sub-block
// links with binary lifting over window minima: ml[k] / mr[k] = the minimum of the 2^k lanes
// ending / starting at this lane, and (pl, lane) extends while its minimum stays >= v.  Only the workgroup's own prefix /
// suffix minima (≈ 2 ln 4096 ≈ 17 of 4,096) go to the global min tree: 64× fewer dependent
// global searches than one wave per 64 ranks.
constexpr uint32_t kAnsvBlock = 4096, kAnsvSub = kAnsvBlock / 64;
constexpr uint16_t kNone16 = 0xffffu;    // (block-local indices are < 4,096)
constexpr uint16_t kQueued16 = 0xc000u;  // | queue slot: resolved through the global min tree
constexpr uint32_t kAnsvQCap = 512;      // (a random block has ≈ 2 ln 4096 ≈ 17 such sides)
__global__ void __launch_bounds__(512) k_psa_ansv_blk(uint32_t N, MinTree t, const PsaShard *shards, uint32_t nshards,
                                                      uint2 *links) {
    __shared__ uint32_t V[kAnsvBlock];        // the block's suffix-array values
    __shared__ uint16_t PS[kAnsvBlock], NS[kAnsvBlock];  // block-local index of the nearest smaller, or kNone16
    __shared__ uint32_t M[kAnsvSub];          // sub-block minima
    __shared__ uint16_t Q[kAnsvQCap];         // queued sides: block-local index | dir << 15
    __shared__ uint32_t QR[kAnsvQCap], qn;    // their nearest smaller rank (or kNoPos)
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t b0 = blockIdx.x * kAnsvBlock;
    if (b0 >= N) return;
    const uint32_t *sa = t.lvl[0];
    if (threadIdx.x == 0) qn = 0;
    // phase 1: sub-blocks by lifting
    for (uint32_t sb = wave; sb < kAnsvSub; sb += nw) {
        const uint32_t li = sb * 64 + lane, r = b0 + li;
        const uint32_t v = r < N ? sa[r] : kNoPos;
        uint32_t ml[6], mr[6];
        ml[0] = mr[0] = v;
        for (int k = 1; k < 6; ++k) {
            const uint32_t w = 1u << (k - 1);
            const uint32_t a = (uint32_t)__shfl((int)ml[k - 1], (int)((lane - w) & 63u));
            const uint32_t b = (uint32_t)__shfl((int)mr[k - 1], (int)((lane + w) & 63u));
            ml[k] = lane >= w ? min(ml[k - 1], a) : ml[k - 1];
            mr[k] = lane + w < 64 ? min(mr[k - 1], b) : mr[k - 1];
        }
        int pl = (int)lane - 1, pr = (int)lane + 1;
        for (int k = 5; k >= 0; --k) {
            const int w = 1 << k;
            const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(max(pl, 0) << 2, (int)ml[k]);
            if (pl - w + 1 >= 0 && a >= v) pl -= w;
            const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(min(pr, 63) << 2, (int)mr[k]);
            if (pr + w - 1 <= 63 && b >= v) pr += w;
        }
        V[li] = v;
        PS[li] = pl >= 0 ? (uint16_t)(sb * 64 + (uint32_t)pl) : kNone16;
        NS[li] = pr <= 63 ? (uint16_t)(sb * 64 + (uint32_t)pr) : kNone16;
        // the sub-block's minimum: lanes 0..31 (lane 0's mr[5]) and 32..63 (lane 63's ml[5])
        const uint32_t m63 = (uint32_t)__shfl((int)ml[5], 63);
        if (lane == 0) M[sb] = min(mr[5], m63);
    }
    __syncthreads();
    // phase 2: across sub-blocks, inside the workgroup (LDS only)
    for (uint32_t sb = wave; sb < kAnsvSub; sb += nw) {
        const uint32_t li = sb * 64 + lane;
        const uint32_t v = V[li];
        uint64_t need = __ballot(b0 + li < N && (PS[li] == kNone16 || NS[li] == kNone16));
        const uint32_t mlane = M[lane];  // (kAnsvSub == 64: one sub-block minimum per lane)
        while (need) {
            const uint32_t l = (uint32_t)__ffsll((long long)need) - 1u;
            need &= need - 1;
            const uint32_t vi = (uint32_t)__shfl((int)v, (int)l);
            const uint32_t e = sb * 64 + l;
            if (PS[e] == kNone16) {  // (uniform: every lane reads the same word)
                const uint64_t ms = __ballot(lane < sb && mlane < vi);
                if (ms) {
                    const uint32_t j = 63u - (uint32_t)__clzll((long long)ms);
                    const uint64_t mv = __ballot(V[j * 64 + lane] < vi);
                    if (lane == 0) PS[e] = (uint16_t)(j * 64 + 63u - (uint32_t)__clzll((long long)mv));
                }
            }
            if (NS[e] == kNone16) {
                const uint64_t ms = __ballot(lane > sb && mlane < vi);
                if (ms) {
                    const uint32_t j = (uint32_t)__ffsll((long long)ms) - 1u;
                    const uint64_t mv = __ballot(V[j * 64 + lane] < vi);
                    if (lane == 0) NS[e] = (uint16_t)(j * 64 + (uint32_t)__ffsll((long long)mv) - 1u);
                }
            }
        }
    }
    __syncthreads();
    // phase 3: the workgroup's own prefix / suffix minima (a side unresolved inside the
    // workgroup has no smaller value there) go to a queue, shared out over all waves, and
    // each searches the global min tree from the workgroup's edge outward; a queue overflow
    // (adversarial input) is searched by the owning wave in phase 4
    for (uint32_t sb = wave; sb < kAnsvSub; sb += nw) {
        const uint32_t li = sb * 64 + lane;
        const bool live = b0 + li < N;
        for (uint32_t dir = 0; dir < 2; ++dir) {
            uint16_t *X = dir == 0 ? PS : NS;
            const bool q = live && X[li] == kNone16;
            const uint64_t m = __ballot(q);
            if (!m) continue;
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&qn, (uint32_t)__popcll(m));
            base = (uint32_t)__shfl((int)base, 0);
            const uint32_t slot = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (q && slot < kAnsvQCap) {
                Q[slot] = (uint16_t)(li | (dir << 15));
                X[li] = (uint16_t)(kQueued16 | slot);
            }
        }
    }
    __syncthreads();
    const uint32_t nq = min(qn, kAnsvQCap);
    for (uint32_t i = wave; i < nq; i += nw) {
        const uint32_t item = Q[i], li = item & 0x7fffu, dir = item >> 15;
        const uint32_t f = tree_find(t, dir == 0 ? b0 : b0 + kAnsvBlock - 1, V[li], (int)dir);
        if (lane == 0) QR[i] = f;
    }
    __syncthreads();
    // phase 4: every rank's links (in rank order; k_psa_links_text moves them to text order)
    for (uint32_t sb = wave; sb < kAnsvSub; sb += nw) {
        const uint32_t li = sb * 64 + lane, r = b0 + li;
        const bool live = r < N;
        const uint32_t v = V[li];
        const uint32_t xp = PS[li], xn = NS[li];
        uint32_t ps = xp == kNone16 ? kNoPos : (xp & kQueued16) == kQueued16 ? QR[xp & 0x3fffu] : b0 + xp;
        uint32_t ns = xn == kNone16 ? kNoPos : (xn & kQueued16) == kQueued16 ? QR[xn & 0x3fffu] : b0 + xn;
        if (ns != kNoPos && ns >= N) ns = kNoPos;
        uint64_t need = __ballot(live && (xp == kNone16 || xn == kNone16));  // (queue overflow only)
        while (need) {
            const uint32_t l = (uint32_t)__ffsll((long long)need) - 1u;
            need &= need - 1;
            const uint32_t vi = (uint32_t)__shfl((int)v, (int)l);
            const uint32_t pi = (uint32_t)__shfl((int)xp, (int)l);
            const uint32_t ni = (uint32_t)__shfl((int)xn, (int)l);
            const uint32_t fp = pi == kNone16 ? tree_find(t, b0, vi, 0) : 0u;
            const uint32_t fn = ni == kNone16 ? tree_find(t, b0 + kAnsvBlock - 1, vi, 1) : 0u;
            if (lane == l) {
                if (pi == kNone16) ps = fp;
                if (ni == kNone16) ns = fn;
            }
        }
        if (!live) continue;
        const PsaShard sh = shards[shard_of_rank(shards, nshards, r)];
        const uint32_t lo = sh.base, hi = sh.base + sh.len;
        const uint32_t pv = ps != kNoPos && ps >= lo ? (ps >= b0 ? V[ps - b0] : sa[ps]) : kNoPos;
        const uint32_t nv = ns != kNoPos && ns < hi ? (ns < b0 + kAnsvBlock ? V[ns - b0] : sa[ns]) : kNoPos;
        links[r] = make_uint2(pv, nv);
    }
}

// the links in text order: one scattered 8-byte read per position instead of two
// scattered 4-byte writes in the ANSV kernel (rank = the inverse suffix array)
__global__ void __launch_bounds__(256) k_psa_links_text(uint32_t N, const uint32_t *rank, const uint2 *links,
                                                        uint32_t *psvp, uint32_t *nsvp) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    const uint2 l = links[rank[p]];
    psvp[p] = l.x;
    nsvp[p] = l.y;
}

// ---------------------------------------------------------------- lcp with those neighbours
// text positions per thread (Kasai-style amortisation): 16 (a multiple of 8; the span starts
// are seeded cooperatively by k_psa_lce_seed).  Longer spans re-fetch their lines: a thread's
// 16-byte step through five per-position arrays leaves each line before it is used up, and
// the lines of all threads in flight do not stay cached (config 3, r04: links + lcp 48.6 /
// 48.4 / 46.8 / 44.4 / 42.7 ms at 256 / 128 / 64 / 32 / 16 positions per thread; PMC at
// 256: 86 GB fetched by k_psa_lce per batch)
constexpr uint32_t kLceSpan = 16;
inline uint32_t lce_span(uint64_t n) {
    if (const char *e = std::getenv("PX_LCE_SPAN")) return (uint32_t)std::max(8, std::atoi(e) / 8 * 8);  // (experiments)
    uint64_t sp = kLceSpan;
    while (sp > 16 && n / sp < (1u << 18)) sp /= 2;
    return (uint32_t)sp;
}

// 8 text bytes from any offset: one unaligned 8-byte load (gfx950 runs in unaligned access
// mode; G is padded by 64 bytes).  (Two aligned loads and a funnel shift doubled the lane
// addresses of the LCE's scattered neighbour reads, which are what bounds it on random text.)
typedef uint64_t u64_ua __attribute__((aligned(1)));
PSA_DEV uint64_t ld8(const uint64_t *G8, uint32_t off) {
    return *(const PX_GAS u64_ua *)((const PX_GAS uint8_t *)G8 + off);
}

#ifndef PX_LCE_STEP
#define PX_LCE_STEP 64
#endif
// 16 text bytes from any offset: one unaligned 16-byte load
typedef uint64_t u64x2_ua __attribute__((ext_vector_type(2), aligned(1)));
PSA_DEV u64x2_ua ld16(const uint64_t *G8, uint32_t off) {
    return *(const PX_GAS u64x2_ua *)((const PX_GAS uint8_t *)G8 + off);
}

PSA_DEV uint32_t lce(const uint64_t *G8, uint32_t p, uint32_t q, uint32_t k, uint32_t lim) {
    // bytes equal from offset k on, up to lim (both suffixes stay inside their docs).  Most
    // comparisons end in their first 8 bytes; one that does not runs on 64 bytes per step, four
    // 16-byte loads per side issued together (a thread entering a template copy compares the
    // copy's length alone, a dependent round trip per step: at 8 and then 32 bytes per step
    // such threads were the tail of a single-instance round's launch).  Reads stay below
    // p + lim + 64 <= N + 64, inside G's 64 bytes of padding.
    if (k >= lim) return lim;
    {
        const uint64_t x = ld8(G8, p + k) ^ ld8(G8, q + k);
        if (x) return min(lim, k + (uint32_t)(__builtin_ctzll(x) >> 3));
        k += 8;
    }
#if PX_LCE_STEP == 32  // (A/B: 32 bytes per step, eight 8-byte loads)
    while (k < lim) {
        const uint64_t a = ld8(G8, p + k) ^ ld8(G8, q + k), b = ld8(G8, p + k + 8) ^ ld8(G8, q + k + 8),
                       c = ld8(G8, p + k + 16) ^ ld8(G8, q + k + 16), d = ld8(G8, p + k + 24) ^ ld8(G8, q + k + 24);
        if (a | b | c | d) {
            const uint32_t o = a ? 0u : b ? 8u : c ? 16u : 24u;
            const uint64_t x = a ? a : b ? b : c ? c : d;
            return min(lim, k + o + (uint32_t)(__builtin_ctzll(x) >> 3));
        }
        k += 32;
    }
    return lim;
#else
    while (k < lim) {
        const u64x2_ua a = ld16(G8, p + k) ^ ld16(G8, q + k), b = ld16(G8, p + k + 16) ^ ld16(G8, q + k + 16),
                       c = ld16(G8, p + k + 32) ^ ld16(G8, q + k + 32), d = ld16(G8, p + k + 48) ^ ld16(G8, q + k + 48);
        const uint64_t w[8] = {a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
        if (w[0] | w[1] | w[2] | w[3] | w[4] | w[5] | w[6] | w[7]) {
            uint32_t o = 0;
            uint64_t x = 0;
            bool f = false;
#pragma unroll
            for (int i = 0; i < 8; ++i)  // (the first nonzero word)
                if (!f && w[i]) {
                    f = true;
                    o = 8u * (uint32_t)i;
                    x = w[i];
                }
            return min(lim, k + o + (uint32_t)(__builtin_ctzll(x) >> 3));
        }
        k += 64;
    }
    return lim;
#endif
}

// The lcp values at every span's first position, where k_psa_lce would start from zero: a
// span that begins inside a long repeat (the 8 KB templates) would otherwise compare it 8
// bytes per step alone.  Here 8 lanes share a comparison, 64 bytes per step; a wave runs
// 8 comparisons (4 span starts, each with both neighbours).  seed[2 t] / seed[2 t + 1] =
// lcp with the previous / next smaller neighbour of span t's first position.
//
// Most span starts need no comparison (round 6): where a neighbour chain continues through the
// whole span before (q = q' + 1 at every position) the shifted-pair identity k_psa_lce uses
// (lcp(p - 1, q') = L >= 2 gives lcp(p, q' + 1) = L - 1 exactly) carries the last computed
// seed S of the chain's run forward: S - span * (t - s) for span t of a run started at span s,
// valid while it stays >= 1 (then every position between had L >= 2).  brk[t] (k_psa_seed_brk)
// is t + 1 where side `side` of span t does not continue span t - 1's chain, else 0; its
// max-scan gives each span its run start.  Launched twice: `derive` 0 compares the runs' first
// spans; `derive` 1 carries their seeds along the runs and compares where that is not valid.
__global__ void __launch_bounds__(256) k_psa_seed_brk(uint32_t N, uint32_t nspan, const uint32_t *psvp,
                                                      const uint32_t *nsvp, uint32_t span, uint32_t *brk_p,
                                                      uint32_t *brk_n) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nspan) return;
    bool cp = t > 0, cn = t > 0;
    if (t > 0) {
        const uint32_t p0 = t * span, a = p0 - span;
        uint32_t qp = psvp[a], qn = nsvp[a];
        cp = qp != kNoPos;
        cn = qn != kNoPos;
        for (uint32_t p = a + 1; p <= p0 && (cp || cn); ++p) {
            const uint32_t xp = psvp[p], xn = nsvp[p];
            cp = cp && xp != kNoPos && xp == qp + 1;
            cn = cn && xn != kNoPos && xn == qn + 1;
            qp = xp;
            qn = xn;
        }
    }
    brk_p[t] = cp ? 0u : t + 1u;
    brk_n[t] = cn ? 0u : t + 1u;
}
__global__ void __launch_bounds__(256) k_psa_lce_seed(uint32_t N, uint32_t nspan, const uint64_t *G8,
                                                      const uint16_t *dist, const uint32_t *psvp,
                                                      const uint32_t *nsvp, uint32_t span, uint16_t *seed,
                                                      const uint32_t *run_p, const uint32_t *run_n, uint32_t derive) {
    const uint32_t lane = lane_id(), grp = lane >> 3, sub = lane & 7u;
    const uint32_t c = (blockIdx.x * blockDim.x + threadIdx.x) >> 3;  // comparison index
    const uint32_t t = c >> 1;
    bool live = t < nspan;
    if (live && run_p) {  // (run_p null: every span compares)
        const uint32_t s = ((c & 1u) ? run_n[t] : run_p[t]) - 1u;  // the run's first span
        if (!derive) {
            live = s == t;
        } else if (s == t) {
            live = false;  // (compared by the first launch)
        } else {
            const uint32_t S = seed[2 * s + (c & 1u)];
            const uint64_t d = (uint64_t)span * (t - s);
            if ((uint64_t)S >= d + 1) {
                if (sub == 0) seed[c] = (uint16_t)(S - d);
                live = false;
            }
        }
    }
    uint32_t p = 0, q = kNoPos, lim = 0;
    if (live) {
        p = t * span;
        q = (c & 1u) ? nsvp[p] : psvp[p];
        if (q != kNoPos) lim = min((uint32_t)dist[p], (uint32_t)dist[q]);
    }
    uint32_t res = lim;  // (kNoPos: 0)
    bool done = !live || q == kNoPos;
    for (uint32_t k = 0;; k += 64) {
        done = done || k >= lim;
        if (!__ballot(!done)) break;
        const uint32_t off = k + 8 * sub;
        uint64_t x = 0;
        if (!done && off < lim) x = ld8(G8, p + off) ^ ld8(G8, q + off);
        const uint64_t m = __ballot(x != 0);
        const uint32_t gm = (uint32_t)(m >> (8 * grp)) & 0xffu;
        if (!done && gm) {
            const uint32_t first = (uint32_t)__ffs(gm) - 1u;  // the group's first mismatching lane
            const uint64_t xf = shfl64(x, grp * 8 + first);
            res = min(lim, k + 8 * first + (uint32_t)(__builtin_ctzll(xf) >> 3));
            done = true;
        }
    }
    if (live && sub == 0) seed[c] = (uint16_t)(q == kNoPos ? 0u : res);
}

// One thread per `span` consecutive positions.  The per-position arrays are read and
// written 8 positions at a time with 16-byte accesses: a wave's 64 threads sit 256
// positions apart, so per-position 2- and 4-byte accesses would each touch a different
// cache line (and 64 threads x 5 arrays of such lines do not stay cached between the
// thread's consecutive positions).
__global__ void __launch_bounds__(256) k_psa_lce(uint32_t N, const uint64_t *G8, const uint16_t *dist,
                                                 const uint32_t *psvp, const uint32_t *nsvp, uint16_t *lcp_p,
                                                 uint16_t *lcp_n, uint32_t span, const uint16_t *seed) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t p0 = t * span;
    if (p0 >= N) return;
    const uint32_t seed_p = seed[2 * t], seed_n = seed[2 * t + 1];
    const uint32_t p1 = min(N, p0 + span);
    uint32_t kp = 0, kn = 0, qprev = kNoPos - 1, sprev = kNoPos - 1;
    for (uint32_t b = p0; b < p1; b += 8) {
        const uint32_t nb = min(8u, p1 - b);
        // (register arrays: every index below is a compile-time constant)
        uint32_t dv[8], qv[8], sv[8], op[4] = {0, 0, 0, 0}, on[4] = {0, 0, 0, 0};
        if (nb == 8) {  // b is a multiple of 8: aligned vector loads
            const uint4 d4 = *(const uint4 *)(dist + b);
            const uint4 qa = *(const uint4 *)(psvp + b), qb = *(const uint4 *)(psvp + b + 4);
            const uint4 sa = *(const uint4 *)(nsvp + b), sb = *(const uint4 *)(nsvp + b + 4);
            const uint32_t dw[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) dv[i] = (dw[i >> 1] >> (16u * (i & 1u))) & 0xffffu;
            qv[0] = qa.x, qv[1] = qa.y, qv[2] = qa.z, qv[3] = qa.w, qv[4] = qb.x, qv[5] = qb.y, qv[6] = qb.z, qv[7] = qb.w;
            sv[0] = sa.x, sv[1] = sa.y, sv[2] = sa.z, sv[3] = sa.w, sv[4] = sb.x, sv[5] = sb.y, sv[6] = sb.z, sv[7] = sb.w;
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) {
                const bool in = i < nb;
                dv[i] = in ? dist[b + i] : 0u;
                qv[i] = in ? psvp[b + i] : kNoPos;
                sv[i] = in ? nsvp[b + i] : kNoPos;
            }
        }
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            if (i < nb) {
                const uint32_t p = b + i, dp = dv[i], q = qv[i], sn = sv[i];
                // the shifted pair: lcp(p-1, q') = L >= 2 gives lcp(p, q'+1) = L - 1 exactly
                // (same mismatch, or the same doc end, one byte on; both stay in their docs),
                // so a neighbour that continues the previous one needs no text at all
                const bool shp = q != kNoPos && q == qprev + 1 && kp >= 2;
                const bool shn = sn != kNoPos && sn == sprev + 1 && kn >= 2;
                kp = kp ? kp - 1 : 0;
                kn = kn ? kn - 1 : 0;
                if (p == p0) {  // (k_psa_lce_seed)
                    kp = seed_p;
                    kn = seed_n;
                } else if (q == kNoPos) {
                    kp = 0;
                } else if (!shp) {
                    const uint32_t lim = min(dp, (uint32_t)dist[q]);
                    kp = lce(G8, p, q, min(kp, lim), lim);
                }
                if (p == p0) {
                } else if (sn == kNoPos) {
                    kn = 0;
                } else if (!shn) {
                    const uint32_t lim = min(dp, (uint32_t)dist[sn]);
                    kn = lce(G8, p, sn, min(kn, lim), lim);
                }
                qprev = q;
                sprev = sn;
                op[i >> 1] |= (kp & 0xffffu) << (16u * (i & 1u));
                on[i >> 1] |= (kn & 0xffffu) << (16u * (i & 1u));
            }
        }
        if (nb == 8) {
            *(uint4 *)(lcp_p + b) = make_uint4(op[0], op[1], op[2], op[3]);
            *(uint4 *)(lcp_n + b) = make_uint4(on[0], on[1], on[2], on[3]);
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) {
                if (i < nb) {
                    lcp_p[b + i] = (uint16_t)(op[i >> 1] >> (16u * (i & 1u)));
                    lcp_n[b + i] = (uint16_t)(on[i >> 1] >> (16u * (i & 1u)));
                }
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
__global__ void __launch_bounds__(256) k_pool_leaf(uint32_t N, const uint8_t *G, const PsaShard *shards, uint32_t nshards,
                                                   const LinkRec *R, uint8_t *code, uint32_t *E, StepStat cs) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t c = 0;
    if (p < N) {
        // (shards are contiguous in position space as in rank space: the same search)
        if (shards[shard_of_rank(shards, nshards, p)].pools) {
            const LinkRec me = R[p];
            const uint32_t l = max(me.lp, me.ln);
            if (l < me.dist) {  // p + l before the doc's end
                c = 1;
                if (l) {
                    uint32_t q = kNoPos;
                    if (me.ln < l) q = me.psv;
                    else if (me.lp < l || R[me.psv].dist == l) q = me.nsv;
                    if (q != kNoPos) {
                        // climb to E = the earliest occurrence of T[q .. q+l), keeping q's record
                        LinkRec rq = R[q], r = rq;
                        uint32_t e = q, steps = 0, hop = 0;
                        for (;;) {
                            if (r.lp >= l) {
                                hop = r.lp;
                                e = r.psv;
                            } else if (r.ln >= l) {
                                hop = r.ln;
                                e = r.nsv;
                            } else {
                                break;
                            }
                            ++steps;
                            r = R[e];
                        }
                        // T[q + l] == T[e + l]: trivially when q is E; after one hop its lcp is
                        // lcp(q, E) itself (both suffixes go on past l: bytes equal iff > l);
                        // after more hops the text decides
                        const bool same = steps == 0 ? true : steps == 1 ? hop > l : G[q + l] == G[e + l];
                        if (r.dist > l && rq.dist > l && same) {
                            c = 2;
                            E[p] = e;
                        }
                    }
                }
            }
        }
        code[p] = (uint8_t)c;
    }
    // the candidate count: one sharded atomic per workgroup (a single counter taking one
    // atomic per wave serialised the launch)
    block_stat(cs, c == 2 ? 1u : 0u, 0, 0);
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

// The same decision without the hash table (default; PX_POOL_HASH=1 selects the table above):
// the candidates in position order (a flag scan), stably sorted by (E, l) -- so each key's run
// starts with its smallest position, the one that splits.  The table's two fabric atomics per
// candidate (device-scope atomics bypass the XCD's L2) were most of a single-instance round's
// pool emulation: k_pool_insert 0.6 ms of its ~1.2 ms.
// candidates per 256 positions (the compaction's scan runs over these, not over every position)
__global__ void __launch_bounds__(256) k_pool_ccount(uint32_t N, const uint8_t *code, uint32_t *bc) {
    __shared__ uint32_t wc[4];
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t m = __ballot(p < N && code[p] == 2);
    if (lane_id() == 0) wc[threadIdx.x >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}
// candidate p -> slot (candidates before its block, from the inclusive scan) + its rank in the block
__global__ void __launch_bounds__(256) k_pool_cpack(uint32_t N, const uint8_t *code, const uint32_t *E, const uint16_t *lp,
                                                    const uint16_t *ln, const uint32_t *bincl, uint64_t *ck, uint32_t *cv) {
    __shared__ uint32_t wc[4];
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x, w = threadIdx.x >> 6;
    const bool c = p < N && code[p] == 2;
    const uint64_t m = __ballot(c);
    if (lane_id() == 0) wc[w] = (uint32_t)__popcll(m);
    __syncthreads();
    if (!c) return;
    uint32_t i = blockIdx.x ? bincl[blockIdx.x - 1] : 0u;
    for (uint32_t x = 0; x < w; ++x) i += wc[x];
    i += (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
    ck[i] = (uint64_t)E[p] << 16 | max(lp[p], ln[p]);
    cv[i] = p;
}
__global__ void __launch_bounds__(256) k_pool_cmark(uint32_t nc, const uint64_t *ck, const uint32_t *cv, uint8_t *code) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nc) return;
    code[cv[i]] = (i == 0 || ck[i - 1] != ck[i]) ? 3 : 1;
}
__global__ void __launch_bounds__(256) k_pool_cblk(uint32_t N, const uint8_t *code, uint32_t *blk) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    const uint32_t c = code[p];
    blk[p] = c == 1 ? 8u : c == 3 ? 16u : 0u;
}

// C[b] = the blocks before the end of the b-th kPoolCoarse-position block
constexpr uint32_t kPoolCoarse = 1024;
__global__ void __launch_bounds__(256) k_pool_coarse(uint32_t N, const uint32_t *P, uint32_t *C) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if ((uint64_t)b * kPoolCoarse >= N) return;
    C[b] = P[min(b * kPoolCoarse + kPoolCoarse - 1, N - 1)];
}

// One block per emulating shard: the pool state from the chunk's root node on, boundary by
// boundary.  A pool boundary is the first leaf whose pattern does not fit the open pool;
// boundaries form one dependent chain (~2,000 per chunk, ~5,500 positions apart), so the
// scan is latency-bound and built to keep HBM off that chain.  The prefix values P are
// staged into LDS in kScanWin-position windows; wave 0 resolves every boundary inside a
// window from LDS (a ballot over 64-position maxima, then one over the 64 positions) and
// charges the leaf's [5, 3] / [5, 5, 3, 3] blocks one by one, while the other 15 waves stage
// the following window into the second buffer.  A boundary further on than that (a long
// stretch of positions without leaves) is found through the 1,024-position coarse values C
// and its window staged by all waves.  The 2,048th pool opened inside doc g rotates the chunk
// before doc g + 1 (PiXiuCtrl.cpp:13); the window's doc count never reaches 65,535 (the host
// rotates slot-full chunks between rounds).
constexpr uint32_t kScanWin = 16384, kScanThreads = 1024;
PSA_DEV void scan_stage(uint32_t *Pw, uint32_t *Cw, const uint32_t *P, uint32_t N, uint32_t wb, uint32_t t0,
                        uint32_t nt) {
    // every load of the window goes out before any LDS store (up to kStageRegs 16-byte
    // loads per thread): one HBM round trip per window, not one per loop step
    constexpr uint32_t kStageRegs = 5;  // (16,384 positions over >= 960 threads)
    uint4 v[kStageRegs];
#pragma unroll
    for (uint32_t r = 0; r < kStageRegs; ++r) {
        const uint32_t i = (t0 + r * nt) * 4;
        if (i >= kScanWin) continue;
        if (wb + i + 4 <= N) {
            v[r] = *(const uint4 *)(P + wb + i);
        } else {  // (0xffffffff past N: "exceeds")
            v[r].x = wb + i < N ? P[wb + i] : 0xffffffffu;
            v[r].y = wb + i + 1 < N ? P[wb + i + 1] : 0xffffffffu;
            v[r].z = wb + i + 2 < N ? P[wb + i + 2] : 0xffffffffu;
            v[r].w = wb + i + 3 < N ? P[wb + i + 3] : 0xffffffffu;
        }
    }
#pragma unroll
    for (uint32_t r = 0; r < kStageRegs; ++r) {
        const uint32_t i = (t0 + r * nt) * 4;
        if (i >= kScanWin) continue;
        *(uint4 *)(Pw + i) = v[r];
        if ((i & 63) == 60) Cw[i >> 6] = v[r].w;  // the 64-position group's last value
    }
}
// first i in [lo, hi) with key(i) > t (key non-decreasing), hi if none: one wave, 64-ary
// narrowing (one dependent load per 64x), every lane calls it
template <class Key>
PSA_DEV uint32_t wave_first_gt(uint32_t lo, uint32_t hi, uint32_t t, Key key) {
    const uint32_t lane = lane_id();
    while (hi - lo > 64) {
        const uint32_t step = (hi - lo + 63) / 64;
        const uint32_t last = min(lo + (lane + 1) * step, hi) - 1;
        const uint64_t m = __ballot(lo + lane * step < hi && key(last) > t);
        if (!m) return hi;
        const uint32_t L = lobit(m);
        hi = min(lo + (L + 1) * step, hi);
        lo = lo + L * step;
    }
    const uint64_t m = __ballot(lo + lane < hi && key(lo + lane) > t);
    return m ? lo + lobit(m) : hi;
}

__global__ void __launch_bounds__(kScanThreads) k_pool_scan(uint32_t nshards, const PsaShard *shards, const PsaDoc *docs,
                                                            const uint32_t *P, const uint32_t *C, uint32_t N,
                                                            PsaPoolOut *out, uint32_t chain_only) {
    __shared__ uint32_t Pw[2][kScanWin];       // P[wb + i]
    __shared__ uint32_t Cw[2][kScanWin / 64];  // P[wb + 64 j + 63]
    __shared__ uint32_t sh_wb, sh_go, sh_restage;
    const uint32_t s = blockIdx.x;
    if (s >= nshards) return;
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    const PsaShard sh = shards[s];
    if (!sh.pools || !sh.ndocs) {
        if (threadIdx.x == 0) out[s] = PsaPoolOut{kNone, 0, 0, 0};
        return;
    }
    const uint32_t nblk = (N + kPoolCoarse - 1) / kPoolCoarse;
    auto S = [&](uint32_t x) { return x ? P[x - 1] : 0u; };  // blocks before position x
    const uint32_t start = docs[sh.doc0].start, endp = sh.base + sh.len;
    // wave 0's state (uniform across its lanes)
    int32_t pools = 1, used = kNodeBlocks;  // the root (SuffixTree::init_prop)
    uint32_t cur = start, base = S(start);
    const uint32_t send = S(endp);
    uint32_t cw = kNone, cv = 0;  // coarse window: blocks [cw, cw + 64)
    uint32_t k_last = kNone;
    auto more = [&]() { return pools < kRotatePools && (uint32_t)used + (send - base) > (uint32_t)kPoolBlocks; };
    // The bound test.  A pool closes when the next charge (<= 5 blocks) does
    // not fit, so pools 1 .. 2,047 each close holding kPoolBlocks - 4 .. kPoolBlocks blocks, and
    // the charge that opens pool 2,048 starts at a running count in [2047 (kPoolBlocks - 4),
    // 2047 kPoolBlocks].  The leaf holding it lies between the first leaf whose running count
    // (root included) passes the low end and the first that passes the high end: if those are
    // in one doc, the chunk rotates before the next doc; if none passes the low end, it does
    // not rotate.  Only the other cases need the boundary chain below.
    if (wave == 0 && !chain_only) {  // (chain_only: PX_DEBUG_POOL_CHAIN, tests of the chain)
        constexpr uint32_t kLo = (uint32_t)(kRotatePools - 1) * (uint32_t)(kPoolBlocks - 4);
        constexpr uint32_t kHi = (uint32_t)(kRotatePools - 1) * (uint32_t)kPoolBlocks;
        // running count through x = kNodeBlocks + (P[x] - base) (P is a modular prefix sum: its
        // differences inside the shard are exact and non-decreasing)
        auto Pk = [&](uint32_t x) { return P[x] - base; };
        const uint32_t klo = wave_first_gt(start, endp, kLo - (uint32_t)kNodeBlocks, Pk);
        uint32_t verdict = 0;  // 0: chain needed, 1: no rotation, 2: rotation before doc rd
        uint32_t rd = kNone;
        if (klo == endp) {
            verdict = 1;
        } else {
            const uint32_t khi = wave_first_gt(klo, endp, kHi - (uint32_t)kNodeBlocks, Pk);
            if (khi != endp) {
                auto Dk = [&](uint32_t g) { return docs[g].start; };
                const uint32_t d0 = sh.doc0, d1 = sh.doc0 + sh.ndocs;
                const uint32_t glo = wave_first_gt(d0, d1, klo, Dk) - 1, ghi = wave_first_gt(d0, d1, khi, Dk) - 1;
                if (glo == ghi) {
                    verdict = 2;
                    rd = glo + 1;
                }
            }
        }
        if (lane == 0) {
            sh_go = verdict;
            if (verdict) out[s] = PsaPoolOut{verdict == 2 ? rd : kNone, verdict == 2 ? kRotatePools : 0, 0, verdict};
        }
    }
    if (threadIdx.x == 0 && chain_only) sh_go = 0;
    __syncthreads();
    if (sh_go) return;  // (uniform: the whole block leaves)
    __syncthreads();
    // the window holding the next boundary (wave 0): from the coarse values
    auto locate = [&]() {
        const uint32_t cap = (uint32_t)(kPoolBlocks - used);
        uint32_t b = cur / kPoolCoarse;  // first b >= cur / kPoolCoarse with C[b] - base > cap
        for (;;) {
            if (cw == kNone || b < cw || b >= cw + 64) {
                cw = b;
                cv = cw + lane < nblk ? C[cw + lane] : 0xffffffffu;
            }
            const uint64_t m = __ballot(cw + lane >= b && (cw + lane >= nblk || cv - base > cap));
            if (m) return cw + (uint32_t)__ffsll((long long)m) - 1u;
            b = cw + 64;
        }
    };
    uint32_t buf = 0, wb = 0;
    if (wave == 0) {
        const uint32_t go = more() ? 1u : 0u;
        if (go) wb = max(locate() * kPoolCoarse, cur & ~63u);
        if (lane == 0) {
            sh_go = go;
            sh_wb = wb;
        }
    }
    __syncthreads();
    if (sh_go) scan_stage(Pw[0], Cw[0], P, N, sh_wb, threadIdx.x, kScanThreads);
    __syncthreads();
    // every window resolves >= 1 boundary or moves on; a window that does neither would
    // loop forever, so a stall ends the scan -- and is reported (how = 3: the host walks the
    // shard instead of trusting a verdict the chain did not reach)
    uint32_t last_cur = kNone;
    bool stalled = false;
    while (sh_go) {
        wb = sh_wb;
        const uint32_t wend = wb + kScanWin;
        if (wave == 0) {
            const uint32_t *pw = Pw[buf], *cwin = Cw[buf];
            const uint32_t before = wb ? P[wb - 1] : 0u;  // P at wb - 1
            while (more()) {
                const uint32_t cap = (uint32_t)(kPoolBlocks - used);
                // the 64-position group holding the boundary, within the window
                uint32_t j = cur > wb ? (cur - wb) >> 6 : 0u, jg = kNone;
                while (j < kScanWin / 64) {
                    const uint32_t jj = j + lane;
                    const uint64_t m = __ballot(jj < kScanWin / 64 && cwin[jj < kScanWin / 64 ? jj : 0] - base > cap);
                    if (m) {
                        jg = j + (uint32_t)__ffsll((long long)m) - 1u;
                        break;
                    }
                    j += 64;
                }
                if (jg == kNone) break;  // past the window
                const uint32_t x = wb + 64 * jg + lane;
                const uint32_t v = pw[64 * jg + lane];
                const uint64_t mk = __ballot(x >= cur && x < endp && v - base > cap);
                if (!mk) break;  // (only past endp: cannot happen while more())
                const uint32_t L = (uint32_t)__ffsll((long long)mk) - 1u;
                const uint32_t k = wb + 64 * jg + L;
                const uint32_t Pk = (uint32_t)__shfl((int)v, (int)L);
                const uint32_t sk = k == start ? base : (k == wb ? before : pw[k - wb - 1]);
                int32_t u = used + (int32_t)(sk - base);
                const bool split = Pk - sk == 16u;
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
                base = Pk;
                k_last = k;
                if (cur >= wend) break;
            }
        } else {  // the next window, speculatively: the one right after this
            scan_stage(Pw[buf ^ 1], Cw[buf ^ 1], P, N, wend, threadIdx.x - 64, kScanThreads - 64);
        }
        __syncthreads();
        if (wave == 0) {
            const bool m = more();
            stalled = m && cur == last_cur;
            uint32_t go = m && !stalled ? 1u : 0u, nwb = wend, re = 0;
            last_cur = cur;
            if (go) {
                const uint32_t b = locate();
                if (b * kPoolCoarse + kPoolCoarse > wend + kScanWin) {  // beyond the staged window
                    nwb = max(b * kPoolCoarse, cur & ~63u);
                    re = 1;
                }
            }
            if (lane == 0) {
                sh_go = go;
                sh_wb = nwb;
                sh_restage = re;
            }
        }
        __syncthreads();
        buf ^= 1;
        if (sh_go && sh_restage) {
            scan_stage(Pw[buf], Cw[buf], P, N, sh_wb, threadIdx.x, kScanThreads);
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) {
        PsaPoolOut o{kNone, 0, 0, 0};
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
        if (stalled) o.how = 3;
        out[s] = o;
    }
}

}  // namespace


#define PSA_CHECK(x)                         \
    do {                                     \
        hipError_t e_ = (x);                 \
        if (e_ != hipSuccess) return e_;     \
    } while (0)

namespace {
// Device scratch borrowed from the runtime's heap and released on every exit, errors and
// exceptions (PxFail from the heap) included.  The heap hands a released block out again
// only to later work on the same stream, so releasing while kernels still use it is safe.
class Scratch {
  public:
    explicit Scratch(const PsaAlloc &A) : A_(A) {}
    Scratch(const Scratch &) = delete;
    ~Scratch() {
        for (auto &b : live_) A_.release(A_.self, b.first, b.second);
    }
    template <class T>
    T *get(uint64_t bytes) {
        void *p = A_.alloc(A_.self, bytes);
        live_.emplace_back(p, bytes);
        return static_cast<T *>(p);
    }
    void put(const void *p) {
        for (size_t i = 0; i < live_.size(); ++i)
            if (live_[i].first == p) {
                A_.release(A_.self, live_[i].first, live_[i].second);
                live_[i] = live_.back();
                live_.pop_back();
                return;
            }
    }

  private:
    const PsaAlloc &A_;
    std::vector<std::pair<void *, uint64_t>> live_;
};
struct EventSet {
    std::vector<hipEvent_t> e;
    ~EventSet() {
        for (auto x : e) (void)hipEventDestroy(x);
    }
    hipError_t make(size_t n, unsigned flags) {
        while (e.size() < n) {
            hipEvent_t x;
            const hipError_t r = hipEventCreateWithFlags(&x, flags);
            if (r != hipSuccess) return r;
            e.push_back(x);
        }
        return hipSuccess;
    }
};
bool env_on(const char *name) {
    const char *v = std::getenv(name);
    return v && *v == '1';
}
constexpr uint32_t kPinUnset = 0xffffffffu;  // a late step's pinned count not yet written
constexpr uint32_t kMaxSteps = 20;  // h doubles from >= 5 past 65,535 (the longest doc) in 15
// persistent grids of the doubling kernels (grid-stride over windows, and over lists whose
// sizes only the device knows)
constexpr uint32_t kGridWin = 16384, kGridReg = 2048, kGridBlk = 1024;
// the cnt words of psa_run
constexpr uint32_t kCntLong = 0, kCntSorted = 16, kCntActive = 48, kCntMax = 96, kCntCand = 200, kCntSortErr = 250,
                   kCntRet = 252, kCntWords = 256;
static_assert(kCntSorted + kMaxSteps < kCntActive && kCntActive + kMaxSteps + 1 < kCntMax && kCntMax + kMaxSteps + 1 < kCntCand, "cnt layout");
}  // namespace

// Runs the pipeline; messages land in every new doc's msg array, the new records' chunk /
// slot / status in rec_*, and shard_flag[k] (device, zeroed by the caller) is set for shards
// whose stream may differ from the reference's (walk them with k_gst_encode instead).
// With any_pools, the shards marked `pools` get the MemPool emulation: pool_out[k] (device)
// says where shard k's live chunk rotates inside this window (see k_pool_scan).
hipError_t psa_run(hipStream_t s, const PsaAlloc &A, uint32_t ndocs, const PsaDoc *docs, uint32_t nshards,
                   const PsaShard *shards, const PsaShard *hshards, uint32_t N, uint32_t *rec_chunk, uint32_t *rec_idx, uint32_t *rec_status,
                   uint32_t *shard_flag, bool any_pools, PsaPoolOut *pool_out, PsaStats *st) {
    if (!N || !ndocs) return hipSuccess;
    if (nshards > kPsaMaxShards) return hipErrorInvalidValue;  // (the caller splits rounds below this)
    Scratch S(A);
    EventSet ev, sev;
    PSA_CHECK(ev.make(5, hipEventDefault));
    hipEvent_t e0 = ev.e[0], e1 = ev.e[1], e2 = ev.e[2], e3 = ev.e[3], e4 = ev.e[4];
    const bool verbose = env_on("PX_PSA_VERBOSE");
    PSA_CHECK(hipEventRecord(e0, s));
    const uint64_t n64 = N;
    const uint32_t tb = 256;
    auto blocks = [&](uint64_t n) { return (uint32_t)((n + tb - 1) / tb); };
    auto *G = S.get<uint8_t>(n64 + 64);
    auto *pdoc = S.get<uint32_t>(n64 * 4);
    auto *dist = S.get<uint16_t>(n64 * 2);
    auto *rank = S.get<uint32_t>(n64 * 4);
    auto *sa = S.get<uint32_t>(n64 * 4);
    // cnt: counters read back by the host (kCnt* offsets)
    auto *cnt = S.get<uint32_t>(kCntWords * 4);
    uint32_t *ncand = cnt + kCntCand;
    PSA_CHECK(hipMemsetAsync(G + N, 0, 64, s));  // (ld8 reads up to 15 bytes past the text)
    PSA_CHECK(hipMemsetAsync(cnt, 0, kCntWords * 4, s));

    // ---- first sort: `syms` (6) symbols of 9 bits per suffix, inside each shard (px_sort.hip: the
    // shards are contiguous in position space and their suffix-array ranges are the same
    // ranges, so each shard sorts on its own and no key carries the shard)
    // (PX_PSA_SYMS = 2..6 for tests and measurements: fewer symbols give odd pass counts,
    // which px_route.h routes; more do not fit below the reach bits, kDlShift)
    uint32_t syms = 6;
    if (const char *ev_syms = std::getenv("PX_PSA_SYMS")) syms = (uint32_t)std::min(6, std::max(2, std::atoi(ev_syms)));
    {
        const uint32_t slices = std::max<uint32_t>(1, std::min<uint32_t>(64, 16384 / ndocs));
        const uint64_t nw = (uint64_t)ndocs * slices;
        k_psa_gather<<<(uint32_t)std::min<uint64_t>((nw + 3) / 4, 65535u), 256, 0, s>>>(ndocs, docs, slices, G, pdoc, dist);
    }
    const SortAlloc SA{A.alloc, A.release, A.self};
    auto *keys = S.get<uint64_t>(n64 * 8);
    auto *keys2 = S.get<uint64_t>(n64 * 8);  // (the sorted keys: the first grouping reads their reach)
    {
        std::vector<uint32_t> slen(nshards);
        for (uint32_t i = 0; i < nshards; ++i) slen[i] = hshards[i].len;
        auto *segs = S.get<uint32_t>((uint64_t)nshards * 8 + 64);
        k_psa_segs<<<(nshards + 255) / 256, 256, 0, s>>>(nshards, shards, segs, segs + nshards);
        auto *va = S.get<uint32_t>(n64 * 4), *vb = S.get<uint32_t>(n64 * 4);
        // passes: text -> keys -> keys2 -> keys -> keys2 -> keys -> (keys2, sa)
        PSA_CHECK(seg_sort_pairs(s, SA, nshards, seg_tile_count(slen.data(), nshards), segs, segs + nshards, 9 * syms, 9,
                                 nullptr, nullptr, G, dist, syms, keys, va, keys2, vb, keys2, sa, cnt + kCntSortErr));
        S.put(segs);
        S.put(va);
        S.put(vb);
    }
    // ---- the first groups, then prefix doubling over them
    auto *sd = S.get<uint16_t>(n64 * 2);
    auto *act = S.get<uint8_t>(n64 + 64);
    auto *gsz = S.get<uint32_t>(n64 * 4 + 64);
    // step k's counters: suffixes sorted, slots still in groups after it, largest group left
    // (index 0 of active / maxsz: after the first grouping)
    // (region 0: the first grouping, region k + 1: step k)
    auto *stat_sh = S.get<uint32_t>((uint64_t)(kMaxSteps + 1) * kStatShards * kStatStride * 4);
    PSA_CHECK(hipMemsetAsync(stat_sh, 0, (size_t)(kMaxSteps + 1) * kStatShards * kStatStride * 4, s));
    auto region = [&](uint32_t k) { return StepStat{stat_sh + (uint64_t)k * kStatShards * kStatStride}; };
    auto stats_of = [&](uint32_t k) { return region(k + 1); };
    {
        auto *chain = (unsigned long long *)keys;  // (the pass buffers are spent: the look-back chain and its ticket)
        const uint32_t g0 = (uint32_t)((n64 + kG0Slots - 1) / kG0Slots);
        PSA_CHECK(hipMemsetAsync(chain, 0, ((uint64_t)g0 + 1) * 8, s));
        k_psa_groups0<<<g0, 256, 0, s>>>(N, sa, keys2, chain, cnt + kCntSortErr, rank, sd, act, gsz, region(0));
    }
    k_stat_sum<<<1, 64, 0, s>>>(region(0).sh, cnt + kCntSorted + kMaxSteps, cnt + kCntActive, cnt + kCntMax);
    S.put(keys);
    S.put(keys2);
    auto *key = S.get<uint32_t>(n64 * 4 + 64);
    LongLists LL;
    {
        const uint32_t lo[kLongClasses] = {kWinMax + 1, 129, 257, kRegMax + 1, kMedMax + 1};
        for (int c = 0; c < kLongClasses; ++c) {
            LL.cap[c] = (uint32_t)(n64 / lo[c] + 64);
            LL.lst[c] = S.get<uint64_t>((uint64_t)LL.cap[c] * 8);
        }
        LL.cnt = cnt + kCntLong;
    }
    // retired groups (see RetList; off unless PX_PSA_RETIRE=1: measured on config 3 they take
    // 6 ms off the window sorter but add 4 ms of link walks to the key gathers and 11 ms of
    // resolution, CHANGELOG.md round 5): list capped at N / 32 (groups past it stay in the doubling)
    RetList R{};
    if (env_on("PX_PSA_RETIRE")) {
        R.per = (uint32_t)std::min<uint64_t>((n64 / 32 + 4096) / kRetShards + 1, 0x7fffffffull / kRetShards);
        R.cap = R.per * kRetShards;
        R.ent = S.get<uint4>((uint64_t)R.cap * 16);
        R.lnk = S.get<unsigned long long>((uint64_t)R.cap * 8);
        R.sc = S.get<uint32_t>(kRetShards * kRetStride * 4);
        PSA_CHECK(hipMemsetAsync(R.sc, 0, kRetShards * kRetStride * 4, s));
        R.cnt = cnt + kCntRet;
        R.n = N;
    }
    const uint32_t gret = std::min<uint32_t>((R.cap + 255) / 256, 2048);
    uint32_t *pin = A.pin;  // pinned host words: counts come back through them
    auto read_words = [&](uint32_t at, uint32_t n) -> hipError_t {  // -> pin[at .. at + n)
        hipError_t e = hipMemcpyAsync(pin + at, cnt + at, n * 4, hipMemcpyDeviceToHost, s);
        return e == hipSuccess ? hipStreamSynchronize(s) : e;
    };
    PSA_CHECK(read_words(0, kCntWords));
    uint32_t active = pin[kCntActive], maxsz = pin[kCntMax];
    uint32_t h = syms, it = 0;
    // (k_dbl_win: one wave per 64-window chunk at most -- a single-instance round of 12 M positions
    // has 3,076 chunks, and 16,384 workgroups of which 15,600 had nothing to do cost each of its
    // 636 launches their dispatch)
    const uint64_t nchunk = ((n64 + 63) / 64 + 63) / 64;
    // (chunks shared by up to 8 waves while there are fewer than 16,384 of them)
    uint32_t wsplit = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8, 16384 / std::max<uint64_t>(1, nchunk)));
    if (const char *e = std::getenv("PX_WIN_SPLIT")) wsplit = (uint32_t)std::min(8, std::max(1, std::atoi(e)));  // (A/B)
    const uint32_t gwin = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nchunk * wsplit + 3) / 4, kGridWin));
    // one step: every group's keys (flat), then every group sorted by them (windows, then
    // the long-group lists the window kernel filled); big groups need their count on the host
    // lists: launch the register and LDS sorters (false once every group fits a window: groups
    // only split, so a step whose input's largest group is <= kWinMax fills no list)
    // the big groups' sort keys: ranks relative to their shard, at most the largest shard's length
    uint32_t rel_bits = 1;
    {
        uint32_t maxlen = 1;
        for (uint32_t i = 0; i < nshards; ++i) maxlen = std::max(maxlen, hshards[i].len);
        while (rel_bits < 32 && (maxlen >> rel_bits) != 0) ++rel_bits;
    }
    auto step = [&](bool big, bool lists = true, uint32_t *h_active = nullptr, uint32_t *h_max = nullptr) -> hipError_t {
        const uint32_t tag = (it & 1u) ? kTag : 0u;
        const StepStat ss = stats_of(it);
        hipError_t e = hipSuccess;
        // (one thread per 16-slot piece; a bounded grid striding over the pieces measured slower
        // in the dense steps (29.4 -> 34.1 ms) and no faster when used only in the sparse ones)
        k_dbl_key<<<blocks((n64 + 15) / 16), tb, 0, s>>>(N, h, it, act, sa, sd, rank, key, cnt + kCntLong, R,
                                                          cnt + kCntSortErr);
        k_dbl_win<<<gwin, 256, 0, s>>>(N, tag, h, sa, sd, act, gsz, key, rank, LL, ss, R, wsplit);
        if (lists || big) {
            k_dbl_reg<2><<<kGridReg, 256, 0, s>>>(LL.lst[0], LL.cnt + 0, tag, h, sa, sd, act, gsz, key, rank, ss, R);
            k_dbl_reg<4><<<kGridReg, 256, 0, s>>>(LL.lst[1], LL.cnt + 1, tag, h, sa, sd, act, gsz, key, rank, ss, R);
            k_dbl_reg<8><<<kGridReg, 256, 0, s>>>(LL.lst[2], LL.cnt + 2, tag, h, sa, sd, act, gsz, key, rank, ss, R);
            // (513..4096: the LDS sorter.  A 16-per-lane register sorter for 513..1024 measured slower:
            // 253 VGPRs, one wave per SIMD -- k_dbl_reg + k_dbl_blk 39.0 against 29.6 ms on config 3,
            // profiles/r06d_reg16_ab.txt)
            k_dbl_blk<<<kGridBlk, 256, 0, s>>>(LL.lst[3], LL.cnt + 3, tag, h, sa, sd, act, gsz, key, rank, ss, R);
        }
        auto sum = [&]() {
            k_stat_sum<<<1, 64, 0, s>>>(ss.sh, cnt + kCntSorted + it, cnt + kCntActive + 1 + it, cnt + kCntMax + 1 + it,
                                        h_active, h_max);
        };
        if (big) {
            e = read_words(kCntLong, 8);
            if (e != hipSuccess) return e;
            const uint32_t nbig = pin[kCntLong + kBigClass];
            if (pin[kCntLong + kLongClasses]) return hipErrorUnknown;  // (list overflow: cannot happen)
            if (nbig) {
                std::vector<uint64_t> bl(nbig);
                e = hipMemcpy(bl.data(), LL.lst[kBigClass], (size_t)nbig * 8, hipMemcpyDeviceToHost);  // (synchronous)
                if (e != hipSuccess) return e;
                std::vector<uint32_t> boff(nbig);
                uint64_t T = 0;
                for (uint32_t b = 0; b < nbig; ++b) {
                    boff[b] = (uint32_t)T;
                    T += bl[b] >> 32;
                }
                auto *d_boff = S.get<uint32_t>((uint64_t)nbig * 4 + 64);
                e = hipMemcpy(d_boff, boff.data(), (size_t)nbig * 4, hipMemcpyHostToDevice);
                if (e != hipSuccess) return e;
                auto *ck = S.get<uint64_t>(T * 8), *ck2 = S.get<uint64_t>(T * 8), *cka = S.get<uint64_t>(T * 8);
                auto *cv = S.get<uint32_t>(T * 4), *cv2 = S.get<uint32_t>(T * 4), *cva = S.get<uint32_t>(T * 4);
                auto *gp = S.get<uint32_t>(T * 4), *hf = S.get<uint32_t>(T * 4);
                auto *gd = S.get<uint16_t>(T * 2 + 64);
                const bool packed = nbig <= 0x10000u;
                if (packed)
                    k_big_gather<true><<<blocks(T), tb, 0, s>>>((uint32_t)T, nbig, LL.lst[kBigClass], d_boff, sa, sd, key, ck, cv,
                                                                gp, gd, ss, shards, nshards);
                else
                    k_big_gather<false><<<blocks(T), tb, 0, s>>>((uint32_t)T, nbig, LL.lst[kBigClass], d_boff, sa, sd, key, ck, cv,
                                                                 gp, gd, ss, shards, nshards);
                // every group sorted by its 32-bit keys on its own (px_sort.hip): segments = groups
                std::vector<uint32_t> glen(nbig);
                for (uint32_t b = 0; b < nbig; ++b) glen[b] = (uint32_t)(bl[b] >> 32);
                auto *d_glen = S.get<uint32_t>((uint64_t)nbig * 4 + 64);
                k_big_segs<<<(nbig + 255) / 256, 256, 0, s>>>(nbig, LL.lst[kBigClass], d_glen);
                e = seg_sort_pairs(s, SA, nbig, seg_tile_count(glen.data(), nbig), d_boff, d_glen, rel_bits, 8, ck, cv, nullptr,
                                   nullptr, 0, cka, cva, nullptr, nullptr, ck2, cv2, cnt + kCntSortErr);
                S.put(d_glen);
                if (e != hipSuccess) return e;
                {
                    const uint32_t gb = (uint32_t)((T + kG0Slots - 1) / kG0Slots);
                    auto *chain = (unsigned long long *)hf;  // (hf: 4 T bytes, the chain needs 8 (gb + 1))
                    e = hipMemsetAsync(chain, 0, ((uint64_t)gb + 1) * 8, s);
                    if (e != hipSuccess) return e;
                    if (packed)
                        k_big_place<true><<<gb, 256, 0, s>>>((uint32_t)T, LL.lst[kBigClass], d_boff, ck2, cv2, gp, gd, tag, chain,
                                                             cnt + kCntSortErr, sa, sd, act, gsz, rank, ss);
                    else
                        k_big_place<false><<<gb, 256, 0, s>>>((uint32_t)T, LL.lst[kBigClass], d_boff, ck2, cv2, gp, gd, tag, chain,
                                                              cnt + kCntSortErr, sa, sd, act, gsz, rank, ss);
                }
                for (const void *q : {(const void *)d_boff, (const void *)ck, (const void *)ck2, (const void *)cv,
                                      (const void *)cv2, (const void *)gp, (const void *)hf, (const void *)gd,
                                      (const void *)cka, (const void *)cva})
                    S.put(q);
            }
        }
        sum();
        ++it;
        h *= 2;
        return hipGetLastError();
    };
    // host-driven while a group may exceed kMedMax (its radix sort needs the host); groups
    // only split, so afterwards the steps run without host round trips: the host stays one
    // step ahead and stops one (empty, cheap) step after the last group
    while (active > 0 && maxsz > kMedMax) {
        if (it >= kMaxSteps) return hipErrorUnknown;  // cannot happen: docs are <= 65,535 bytes
        PSA_CHECK(step(true));
        PSA_CHECK(read_words(0, kCntWords));
        active = pin[kCntActive + it];
        maxsz = pin[kCntMax + it];
        if (verbose)
            fprintf(stderr, "psa: step %u (host) sorted %u (long groups %u %u %u %u %u) -> %u in groups, largest %u\n",
                    it - 1, pin[kCntSorted + it - 1], pin[kCntLong], pin[kCntLong + 1], pin[kCntLong + 2],
                    pin[kCntLong + 3], pin[kCntLong + 4], active, maxsz);
    }
    if (active > 0) {
        PSA_CHECK(sev.make(kMaxSteps, hipEventDisableTiming));
        const uint32_t it0 = it;
        bool done = false;
        // (pin[256 + k] / pin[288 + k]: slots in groups / the largest group after step k, known on the
        // host once step k's event has passed -- two steps behind the step being enqueued)
        uint32_t known_max = maxsz;  // the largest group after the last step whose counts are back
        while (!done) {
            if (it >= kMaxSteps) return hipErrorUnknown;
            // (k_stat_sum writes step k's counts into pin[256 + k] / pin[288 + k] itself)
            static const bool pin_copy = env_on("PX_PIN_COPY");  // (A/B: the counts copied back)
            // (a sentinel first: a count the kernel's store has not yet made visible reads as the
            // sentinel, never as a stale value, and is then fetched from the device -- a stale
            // nonzero count had the host enqueue empty steps up to kMaxSteps, 90-260 ms, r06fin2)
            pin[256 + it] = kPinUnset;
            pin[288 + it] = kPinUnset;
            PSA_CHECK(step(false, known_max > kWinMax, pin_copy ? nullptr : pin + 256 + it, pin_copy ? nullptr : pin + 288 + it));
            const uint32_t k = it - 1;
            if (pin_copy) {
                PSA_CHECK(hipMemcpyAsync(pin + 256 + k, cnt + kCntActive + 1 + k, 4, hipMemcpyDeviceToHost, s));
                PSA_CHECK(hipMemcpyAsync(pin + 288 + k, cnt + kCntMax + 1 + k, 4, hipMemcpyDeviceToHost, s));
            }
            PSA_CHECK(hipEventRecord(sev.e[k], s));
            if (k >= it0 + 1) {
                PSA_CHECK(hipEventSynchronize(sev.e[k - 1]));
                uint32_t got[2] = {__atomic_load_n(pin + 256 + k - 1, __ATOMIC_ACQUIRE),
                                   __atomic_load_n(pin + 288 + k - 1, __ATOMIC_ACQUIRE)};
                if (got[0] == kPinUnset || got[1] == kPinUnset) {  // (not visible yet: the device's own words)
                    PSA_CHECK(hipMemcpy(&got[0], cnt + kCntActive + 1 + (k - 1), 4, hipMemcpyDeviceToHost));
                    PSA_CHECK(hipMemcpy(&got[1], cnt + kCntMax + 1 + (k - 1), 4, hipMemcpyDeviceToHost));
                }
                done = got[0] == 0;
                known_max = got[1];
            }
        }
    }
    if (R.ent) {  // the retired groups' final order (every live suffix's rank is final now)
        // pointer jumping until no link changes (a template's same-step chain: log2 of its length)
        auto *lnk2 = S.get<unsigned long long>((uint64_t)R.cap * 8);
        unsigned long long *a = R.lnk, *b = lnk2;
        for (uint32_t round = 0; round < 32; ++round) {
            PSA_CHECK(hipMemsetAsync(cnt + kCntRet + 2, 0, 4, s));
            k_ret_jump<<<gret, 256, 0, s>>>(R, a, b, rank);
            std::swap(a, b);
            PSA_CHECK(read_words(kCntRet, 4));
            if (pin[kCntRet + 2] == 0) break;
        }
        RetList Rf = R;
        Rf.lnk = a;
        const uint32_t gw = std::min<uint32_t>((R.cap + 3) / 4, 8192);
        k_ret_resolve<0><<<gw, 256, 0, s>>>(Rf, sa, rank, key, gsz);
        k_ret_resolve<1><<<gw, 256, 0, s>>>(Rf, sa, rank, key, gsz);
        k_ret_resolve<2><<<gw, 256, 0, s>>>(Rf, sa, rank, key, gsz);
    }
    PSA_CHECK(read_words(0, kCntWords));
    if (pin[kCntActive + it] != 0 || pin[kCntLong + kLongClasses] || pin[kCntSortErr] || pin[kCntRet + 1])
        return hipErrorUnknown;
    if (verbose && R.ent) {
        std::vector<uint32_t> sc(kRetShards * kRetStride);
        PSA_CHECK(hipMemcpy(sc.data(), R.sc, sc.size() * 4, hipMemcpyDeviceToHost));
        uint64_t nr = 0;
        for (uint32_t k = 0; k < kRetShards; ++k) nr += std::min(sc[k * kRetStride], R.per);
        fprintf(stderr, "psa: %llu groups retired (list %u)\n", (unsigned long long)nr, R.cap);
    }
    for (const void *q : {(const void *)sd, (const void *)act, (const void *)gsz, (const void *)key}) S.put(q);
    for (int c = 0; c < kLongClasses; ++c) S.put(LL.lst[c]);
    PSA_CHECK(hipEventRecord(e1, s));

    // ---- nearest smaller positions in suffix-array order (min tree over sa)
    MinTree t{};
    t.lvl[0] = sa;
    t.n[0] = N;
    t.levels = 1;
    auto *lv_buf = S.get<uint32_t>(n64 / 64 * 4 * 2 + 1024);
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
    auto *psvp = S.get<uint32_t>(n64 * 4), *nsvp = S.get<uint32_t>(n64 * 4);
    {
        auto *links = S.get<uint2>(n64 * 8);
        k_psa_ansv_blk<<<(uint32_t)((n64 + kAnsvBlock - 1) / kAnsvBlock), 512, 0, s>>>(N, t, shards, nshards, links);
        k_psa_links_text<<<blocks(N), tb, 0, s>>>(N, rank, links, psvp, nsvp);
        S.put(links);
    }
    S.put(lv_buf);
    S.put(sa);
    auto *lcp_p = (uint16_t *)rank;  // ranks are no longer needed: two u16 arrays in their place
    auto *lcp_n = S.get<uint16_t>(n64 * 2);
    const uint32_t lsp = lce_span(n64);
    {
        const uint32_t nspan = (uint32_t)((n64 + lsp - 1) / lsp);
        auto *seed = S.get<uint16_t>((uint64_t)nspan * 4 + 64);
        const uint32_t gseed = (uint32_t)(((uint64_t)nspan * 16 + 255) / 256);
        if (env_on("PX_LCE_SEED_ALL")) {  // (A/B: every span start compared)
            k_psa_lce_seed<<<gseed, 256, 0, s>>>(N, nspan, (const uint64_t *)G, dist, psvp, nsvp, lsp, seed, nullptr,
                                                 nullptr, 0);
        } else {
            auto *brk = S.get<uint32_t>((uint64_t)nspan * 8 + 64);
            uint32_t *brk_p = brk, *brk_n = brk + nspan;
            k_psa_seed_brk<<<blocks(nspan), tb, 0, s>>>(N, nspan, psvp, nsvp, lsp, brk_p, brk_n);
            PSA_CHECK(scan_u32(s, SA, brk_p, brk_p, nspan, ScanOp::kMax, false));
            PSA_CHECK(scan_u32(s, SA, brk_n, brk_n, nspan, ScanOp::kMax, false));
            for (uint32_t derive = 0; derive < 2; ++derive)
                k_psa_lce_seed<<<gseed, 256, 0, s>>>(N, nspan, (const uint64_t *)G, dist, psvp, nsvp, lsp, seed, brk_p,
                                                     brk_n, derive);
            S.put(brk);
        }
        k_psa_lce<<<blocks(nspan), tb, 0, s>>>(N, (const uint64_t *)G, dist, psvp, nsvp, lcp_p, lcp_n, lsp, seed);
        S.put(seed);
    }
    PSA_CHECK(hipEventRecord(e2, s));
    // ---- messages
    k_psa_msg0<<<blocks(N), tb, 0, s>>>(N, pdoc, docs, lcp_p, lcp_n);
    k_psa_runs<<<blocks(N), tb, 0, s>>>(N, G, pdoc, docs, dist, psvp, nsvp, lcp_p, lcp_n, shard_flag);
    k_psa_place<<<blocks(ndocs), tb, 0, s>>>(ndocs, docs, shards, rec_chunk, rec_idx, rec_status);
    PSA_CHECK(hipEventRecord(e3, s));
    if (any_pools) {  // ---- MemPool emulation (rotation points)
        auto *code = S.get<uint8_t>(n64 + 64);
        auto *E = S.get<uint32_t>(n64 * 4), *blk = S.get<uint32_t>(n64 * 4), *P = S.get<uint32_t>(n64 * 4);
        {
            auto *rec = S.get<LinkRec>(n64 * sizeof(LinkRec));
            k_pool_pack<<<blocks(N), tb, 0, s>>>(N, psvp, nsvp, lcp_p, lcp_n, dist, rec);
            auto *csh = S.get<uint32_t>(kStatShards * kStatStride * 4);
            PSA_CHECK(hipMemsetAsync(csh, 0, kStatShards * kStatStride * 4, s));
            k_pool_leaf<<<blocks(N), tb, 0, s>>>(N, G, shards, nshards, rec, code, E, StepStat{csh});
            k_stat_sum<<<1, 64, 0, s>>>(csh, ncand, cnt + kCntCand + 1, cnt + kCntCand + 2);
            S.put(rec);
        }
        // the candidate table: 2x the candidates, read back for big windows; a small window
        // (one chunk, the single instance's rounds) sizes it from N and skips the round trip
        // (sized from the candidate count: one read-back, against a table twice the window
        // that costs a 2x larger clear and spreads the inserts over twice the lines)
        uint32_t nc = 0;
        uint64_t cap = 1024;
        PSA_CHECK(hipMemcpyAsync(pin, ncand, 4, hipMemcpyDeviceToHost, s));
        PSA_CHECK(hipStreamSynchronize(s));
        nc = pin[0];
        if (verbose) fprintf(stderr, "psa pools: %u split candidates\n", nc);
        if (env_on("PX_POOL_HASH")) {  // (the hash-table version, for A/B)
            while (cap < 2ull * nc) cap <<= 1;
            auto *tab = S.get<PoolSlot>(cap * sizeof(PoolSlot));
            PSA_CHECK(hipMemsetAsync(tab, 0xff, cap * sizeof(PoolSlot), s));
            const uint32_t mask = (uint32_t)(cap - 1);
            k_pool_insert<<<blocks(N), tb, 0, s>>>(N, code, E, lcp_p, lcp_n, tab, mask);
            k_pool_blocks<<<blocks(N), tb, 0, s>>>(N, code, E, lcp_p, lcp_n, tab, mask, blk);
        } else {
            if (nc) {
                k_pool_ccount<<<blocks(N), tb, 0, s>>>(N, code, blk);
                PSA_CHECK(scan_u32(s, SA, blk, blk, blocks(N), ScanOp::kPlus, false));
                auto *ck = S.get<uint64_t>((uint64_t)nc * 8), *ck2 = S.get<uint64_t>((uint64_t)nc * 8),
                     *cka = S.get<uint64_t>((uint64_t)nc * 8);
                auto *cv = S.get<uint32_t>((uint64_t)nc * 4), *cv2 = S.get<uint32_t>((uint64_t)nc * 4),
                     *cva = S.get<uint32_t>((uint64_t)nc * 4);
                k_pool_cpack<<<blocks(N), tb, 0, s>>>(N, code, E, lcp_p, lcp_n, blk, ck, cv);
                // one segment [0, nc); keys E << 16 | l below 16 + bit length of N - 1
                auto *seg = S.get<uint32_t>(64);
                PSA_CHECK(hipMemsetAsync(seg, 0, 4, s));
                PSA_CHECK(hipMemcpyAsync(seg + 1, ncand, 4, hipMemcpyDeviceToDevice, s));
                const uint32_t kbits = 16u + (N > 1 ? 32u - (uint32_t)__builtin_clz(N - 1u) : 1u);
                PSA_CHECK(seg_sort_pairs(s, SA, 1, seg_tile_count(&nc, 1), seg, seg + 1, kbits, 8, ck, cv, nullptr, nullptr,
                                         0, cka, cva, nullptr, nullptr, ck2, cv2, cnt + kCntSortErr));
                k_pool_cmark<<<blocks(nc), tb, 0, s>>>(nc, ck2, cv2, code);
                for (const void *q : {(const void *)ck, (const void *)ck2, (const void *)cka, (const void *)cv,
                                      (const void *)cv2, (const void *)cva, (const void *)seg})
                    S.put(q);
            }
            k_pool_cblk<<<blocks(N), tb, 0, s>>>(N, code, blk);
        }
        PSA_CHECK(scan_u32(s, SA, blk, P, N, ScanOp::kPlus, false));
        auto *C = S.get<uint32_t>(n64 / kPoolCoarse * 4 + 256);
        k_pool_coarse<<<blocks((N + kPoolCoarse - 1) / kPoolCoarse), tb, 0, s>>>(N, P, C);
        k_pool_scan<<<nshards, kScanThreads, 0, s>>>(nshards, shards, docs, P, C, N, pool_out,
                                                     env_on("PX_DEBUG_POOL_CHAIN") ? 1u : 0u);
        PSA_CHECK(hipGetLastError());
    }
    PSA_CHECK(hipEventRecord(e4, s));
    PSA_CHECK(hipMemcpyAsync(pin, cnt, kCntWords * 4, hipMemcpyDeviceToHost, s));
    PSA_CHECK(hipEventSynchronize(e4));
    PSA_CHECK(hipStreamSynchronize(s));
    if (st) {
        st->iterations = it;
        for (uint32_t k = 0; k < 24; ++k) st->active[k] = k < kMaxSteps ? pin[kCntSorted + k] : 0;
        st->candidates = any_pools ? pin[kCntCand] : 0;
        PSA_CHECK(hipEventElapsedTime(&st->ms_pool, e3, e4));
        PSA_CHECK(hipEventElapsedTime(&st->ms_sort, e0, e1));
        PSA_CHECK(hipEventElapsedTime(&st->ms_lcp, e1, e2));
        PSA_CHECK(hipEventElapsedTime(&st->ms_msg, e2, e3));
        if (verbose) {
            fprintf(stderr, "psa: N=%u docs=%u shards=%u syms=%u sort %.2f ms, links+lcp %.2f ms, msgs %.2f ms; sorted:",
                    N, ndocs, nshards, syms, st->ms_sort, st->ms_lcp, st->ms_msg);
            for (uint32_t k = 0; k < it && k < 24; ++k) fprintf(stderr, " %u", st->active[k]);
            fprintf(stderr, "\n");
        }
    }
    return hipGetLastError();
}

}  // namespace px
