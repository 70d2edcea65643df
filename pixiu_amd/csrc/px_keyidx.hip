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
//   k_dk_lookup   one thread per query key: probe, verify, pick the span table, out_cap
//   k_dk_fill     output offsets and tile numbers from the two scans, the host's arrays
#include <hip/hip_runtime.h>

#include "px_common.h"

namespace px {
namespace {

#define DK_DEV __device__ __forceinline__

DK_DEV unsigned long long dk_hash(const uint8_t *k, uint32_t n) {
    unsigned long long h = 0x9E3779B97F4A7C15ull ^ n;
    for (uint32_t i = 0; i < n; ++i) {
        h ^= k[i];
        h *= 0x100000001B3ull;
    }
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    return h | 1ull;
}

DK_DEV bool bytes_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i)
        if (a[i] != b[i]) return false;
    return true;
}

__global__ void __launch_bounds__(256) k_dk_insert(uint32_t gid0, uint32_t n, const DkRec *rec, const uint8_t *keys,
                                                   DkSlot *tab, uint32_t mask, uint32_t *err) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t gid = gid0 + j;
    const DkRec r = rec[gid];
    const uint8_t *k = keys + r.key_off;
    const unsigned long long h = dk_hash(k, r.key_len);
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

// per query key: its record's gather query (out_off / tile0 filled by k_dk_fill), its output
// room in 16-byte units and its tiles; a key the index cannot answer counts in *miss
__global__ void __launch_bounds__(256) k_dk_lookup(uint32_t nq, const uint8_t *qkeys, const uint64_t *qoff,
                                                   const DkSlot *tab, uint32_t mask, const DkRec *rec,
                                                   const uint8_t *keys, uint32_t mode, GatherQuery *gq, uint32_t *cap16,
                                                   uint32_t *tiles, uint32_t *miss) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = false;
    if (q < nq) {
        const uint8_t *k = qkeys + qoff[q];
        const uint32_t n = (uint32_t)(qoff[q + 1] - qoff[q]);
        const unsigned long long h = dk_hash(k, n);
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
        uint32_t c16 = 0, nt = 0;
        if (g != kNone) {
            const DkRec r = rec[g];
            const SpanEnt *sp = mode == 0 ? r.sp : r.xsp;
            const uint32_t *t = mode == 0 ? r.t : r.xt;
            const uint32_t ns = mode == 0 ? r.n : r.xn, len = mode == 0 ? r.len : r.xlen;
            if ((r.flags & (kDkLive | kDkClean)) == (kDkLive | kDkClean) && sp) {
                const uint32_t cap = (r.doc_len + 64u + 15u) & ~15u;  // the host's out_cap
                c16 = cap / 16;
                nt = max(1u, (min(len, cap) + kGatherTile - 1) / kGatherTile);
                gq[q] = GatherQuery{sp, r.comp, 0, ns, len, cap, q, t, 0, 0};
                ok = true;
            }
        }
        cap16[q] = c16;
        tiles[q] = nt;
    }
    const unsigned long long m = __ballot(q < nq && !ok);
    if (m && (threadIdx.x & 63u) == 0) atomicAdd(miss, (uint32_t)__popcll(m));
}

// inclusive scans of cap16 / tiles -> every query's output offset and first tile
__global__ void __launch_bounds__(256) k_dk_fill(uint32_t nq, const uint32_t *cap16, const uint32_t *incl_cap16,
                                                 const uint32_t *tiles, const uint32_t *incl_tiles, GatherQuery *gq,
                                                 uint64_t *out_off) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const uint64_t off = (uint64_t)(incl_cap16[q] - cap16[q]) * 16u;
    gq[q].out_off = off;
    gq[q].tile0 = incl_tiles[q] - tiles[q];
    out_off[q] = off;
}

}  // namespace

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
hipError_t launch_dk_lookup(hipStream_t s, uint32_t nq, const uint8_t *qkeys, const uint64_t *qoff, const DkSlot *tab,
                            uint32_t mask, const DkRec *rec, const uint8_t *keys, uint32_t mode, GatherQuery *gq,
                            uint32_t *cap16, uint32_t *tiles, uint32_t *miss) {
    if (!nq) return hipSuccess;
    k_dk_lookup<<<(nq + 255) / 256, 256, 0, s>>>(nq, qkeys, qoff, tab, mask, rec, keys, mode, gq, cap16, tiles, miss);
    return hipGetLastError();
}
hipError_t launch_dk_fill(hipStream_t s, uint32_t nq, const uint32_t *cap16, const uint32_t *incl_cap16,
                          const uint32_t *tiles, const uint32_t *incl_tiles, GatherQuery *gq, uint64_t *out_off) {
    if (!nq) return hipSuccess;
    k_dk_fill<<<(nq + 255) / 256, 256, 0, s>>>(nq, cap16, incl_cap16, tiles, incl_tiles, gq, out_off);
    return hipGetLastError();
}

}  // namespace px
