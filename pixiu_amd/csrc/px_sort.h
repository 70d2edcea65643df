// px_sort.h — hand-written segmented radix sort and u32 scans for the suffix-array pass
// (px_psa.hip).  Host-side entry points; the kernels live in px_sort.hip.
#pragma once
#include <stdint.h>

#include <vector>

#include <hip/hip_runtime.h>

namespace px {

// A tile is kSortTile consecutive elements of ONE segment; a segment's tiles are
// consecutive in the tile table and the first one carries first = 1.
#ifndef PX_SORT_ITEMS
#define PX_SORT_ITEMS 16
#endif
constexpr uint32_t kSortTile = 256 * PX_SORT_ITEMS;
struct SegTile {
    uint32_t start, count, seg, first;
};
// The first sort's keys carry, above their symbols (bits kDlShift..+3), the suffix's doubling
// reach: the number of doubling steps k (h = syms << k) with h < its distance to the doc
// end, i.e. the steps whose key is a rank rather than 0 (<= 14: docs are < 65,536 bytes).
// The sort passes never look at these bits; the first grouping reads them in suffix-array
// order, so the doubling needs no scattered read of the distances.  Keys compare equal on
// their low kKeyBits.
constexpr uint32_t kDlShift = 58, kKeyBits = 54;
constexpr uint64_t kKeyMask = (1ull << kKeyBits) - 1ull;

// device scratch borrowed from the caller (px_psa.hip's Scratch / the runtime heap)
struct SortAlloc {
    void *(*alloc)(void *self, uint64_t n);
    void (*release)(void *self, void *p, uint64_t n);
    void *self;
};

// tiles of segments of these lengths (host)
uint32_t seg_tile_count(const uint32_t *len, uint32_t nseg);

// Stable LSD radix sort of (key, value) pairs inside every segment by key bits [0, bits),
// `rb`-bit digits (8 or 9).  The segments [d_start[g], d_start[g] + d_len[g]) are given on
// the device (ntiles = seg_tile_count of their lengths); the tile table is built there, so
// the sort reads nothing from host memory and never synchronises the stream.  Elements
// never leave their segment, so the scatter of every pass stays inside one segment's range.
// Pass 0 reads (k0, v0), or -- with G / dist set -- computes each position's key from the
// text: `syms` 9-bit symbols (byte + 1, 0 past the doc end; value = the position).  The
// last pass writes (kout, vout).  Scratch pairs: (ka, va) always; (kb, vb) when pass 0 reads
// the text (otherwise k0 / v0 are reused).  Any pass count is routed so that no pass writes a
// buffer it reads (px_route.h); kout / vout may alias kb / vb or k0 / v0.  A pass count that
// cannot be routed returns hipErrorInvalidValue.
// *err (device word, zeroed by the caller) is set if a tile's look-back outlasted its bound
// (cannot happen; the sort is then wrong and the caller must fail).
hipError_t seg_sort_pairs(hipStream_t s, const SortAlloc &A, uint32_t nseg, uint32_t ntiles, const uint32_t *d_start,
                          const uint32_t *d_len, uint32_t bits, int rb, uint64_t *k0, uint32_t *v0, const uint8_t *G,
                          const uint16_t *dist, uint32_t syms, uint64_t *ka, uint32_t *va, uint64_t *kb, uint32_t *vb,
                          uint64_t *kout, uint32_t *vout, uint32_t *err);

enum class ScanOp { kMax, kMin, kPlus };
// inclusive scan of n u32 values (reverse: from the end), in-place allowed
hipError_t scan_u32(hipStream_t s, const SortAlloc &A, const uint32_t *in, uint32_t *out, uint64_t n, ScanOp op,
                    bool reverse);

}  // namespace px
