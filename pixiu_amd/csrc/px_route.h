// px_route.h — which buffers each pass of seg_sort_pairs (px_sort.hip) writes.
//
// A radix pass scatters its input (keys and values) into its output, so no output buffer may
// be an input buffer of the same pass.  The first sort of round 5 routed passes by parity
// (even -> ka, odd -> kb, last -> kout) with kout == kb: a 7-pass (7-symbol) sort then had
// its last pass read and write kb, the in-place scatter corrupted the keys (their doubling
// reach included) and k_dbl_key read rank[p + h] past the round's arrays
// (hipErrorIllegalAddress, gpurun_out/r05d_syms7.log).  sort_route() picks, for any pass
// count, a (keys, values) pair per pass from the ones the caller gave such that no pass
// writes a buffer it reads and the last pass writes (kout, vout), or reports that none
// exists.  Host-only, no HIP: tests/cpp/host_test.cpp checks it for 1..8 passes and the
// aliasings the callers use.
#pragma once
#include <stdint.h>

namespace px {

constexpr uint32_t kRouteMaxPasses = 8;

struct BufPair {
    const void *k, *v;
};
inline bool pair_overlap(const BufPair &a, const BufPair &b) {
    return a.k == b.k || a.v == b.v || a.k == b.v || a.v == b.k;
}

// in0: what pass 0 reads ({nullptr, nullptr} when it computes its keys from the text);
// scratch: up to 4 candidate pairs in order of preference (pairs with a null buffer are
// skipped; the final pair or the input may be among them); fin: the last pass's output.
// On success out[p] is pass p's output for p < passes, out[passes - 1] = fin, and no out[p]
// shares a buffer with pass p's input (in0 for p = 0, out[p - 1] after).
inline bool sort_route(uint32_t passes, BufPair in0, const BufPair scratch[4], BufPair fin,
                       BufPair out[kRouteMaxPasses]) {
    if (passes == 0 || passes > kRouteMaxPasses || !fin.k || !fin.v) return false;
    const uint32_t last = passes - 1;
    if (last == 0) {
        if (pair_overlap(fin, in0)) return false;
        out[0] = fin;
        return true;
    }
    BufPair cand[4];
    uint32_t nc = 0;
    for (uint32_t i = 0; i < 4; ++i)
        if (scratch[i].k && scratch[i].v) cand[nc++] = scratch[i];
    // depth-first over the choices of passes 0 .. passes-2 (<= 4^7 leaves)
    uint32_t pick[kRouteMaxPasses] = {0};
    uint32_t p = 0;
    for (;;) {
        bool ok = false;
        while (pick[p] < nc) {
            const BufPair &b = cand[pick[p]];
            const BufPair &in = p == 0 ? in0 : out[p - 1];
            // (the last intermediate is also the last pass's input, which writes fin)
            if (!pair_overlap(b, in) && (p + 1 < last || !pair_overlap(b, fin))) {
                ok = true;
                break;
            }
            ++pick[p];
        }
        if (ok) {
            out[p] = cand[pick[p]];
            if (p + 1 == last) {
                out[last] = fin;
                return true;
            }
            pick[++p] = 0;
            continue;
        }
        if (p == 0) return false;
        ++pick[--p];
    }
}

}  // namespace px
