// tools/proto/pool_proto.cpp — TEST/DESIGN PROTOTYPE ONLY (never linked into the product).
//
// CPU restatement of the MemPool accounting of the GST walk computed from a suffix array
// (DESIGN.md §9.2), checked against the oracle's Ukkonen walk (pxo_pool_trace).
//
// The walk charges MemPool blocks per created leaf (MemPool.cpp:7-37, SuffixTree.cpp:
// 148-227): a leaf under the root or under an existing node [5, 3] (STNode, child-map
// entry), a leaf that splits an edge [5, 5, 3, 3] (leaf, inner node, two entries).  Leaf j
// of doc D (start s, end e) exists iff j + lpf(j) < e and is created in position order.
// With sigma = T[j .. j+lpf(j)), E = its earliest occurrence and a = T[E + |sigma|]:
//   * sigma is already a node iff an earlier leaf had the same sigma, or E's doc ends right
//     after sigma (E's leaf node);
//   * the leaves with a given sigma are the first occurrences of sigma.c for c != a, so the
//     split happens at the smallest of them: the minimum of the suffix-array interval of
//     sigma outside the interval of sigma.a.  That minimum is the minimum of its side
//     (left or right of sigma.a); a side minimum j has its nearest smaller position on one
//     side outside sigma's interval and on the other inside sigma.a's.  So per sigma at most
//     two candidates exist and the smaller one splits.  Occurrences of sigma that end their
//     doc (sigma.$, sorted first) other than E are implicit suffixes, not leaves: they are
//     skipped (E itself ending its doc is the leaf-node case above).
// extern "C" pool_proto(): pools / used blocks after every doc of one chunk (no rotation).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

namespace {

std::vector<uint32_t> build_sa(const std::vector<uint32_t> &t) {
    const uint32_t n = (uint32_t)t.size();
    std::vector<uint32_t> sa(n), rank(t), tmp(n);
    for (uint32_t i = 0; i < n; ++i) sa[i] = i;
    for (uint32_t h = 1;; h <<= 1) {
        auto key = [&](uint32_t i) { return std::make_pair(rank[i], i + h < n ? rank[i + h] + 1 : 0u); };
        std::sort(sa.begin(), sa.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
        tmp[sa[0]] = 0;
        for (uint32_t r = 1; r < n; ++r) tmp[sa[r]] = tmp[sa[r - 1]] + (key(sa[r - 1]) == key(sa[r]) ? 0 : 1);
        rank = tmp;
        if (tmp[sa[n - 1]] == n - 1) break;
    }
    return sa;
}

struct Pool {
    int32_t pools, used;
    void charge(int32_t b) {
        if (used + b > 65535) {
            ++pools;
            used = b;
        } else {
            used += b;
        }
    }
};

}  // namespace

extern "C" {

// stats: [0] leaves [1] splits [2] one-sided leaves (climbs) [3] climb steps [4] candidates
// [5] longest climb
long pool_proto(int ndocs, const uint8_t *docs, const uint64_t *off, int32_t pools0, int32_t used0, int32_t *pools_out,
                int32_t *used_out, uint64_t *stats) {
    std::vector<uint32_t> t, start(ndocs), end(ndocs), doc_of;
    for (int d = 0; d < ndocs; ++d) {
        start[d] = (uint32_t)t.size();
        for (uint64_t p = off[d]; p < off[d + 1]; ++p) {
            t.push_back((uint32_t)docs[p] + (uint32_t)ndocs);
            doc_of.push_back((uint32_t)d);
        }
        end[d] = (uint32_t)t.size();
        t.push_back((uint32_t)d);  // unique terminator, below every byte (as on the GPU)
        doc_of.push_back((uint32_t)d);
    }
    const uint32_t n = (uint32_t)t.size();
    const std::vector<uint32_t> sa = build_sa(t);
    const uint32_t kNo = 0xffffffffu;
    std::vector<uint32_t> psv(n, kNo), nsv(n, kNo), st;
    for (uint32_t r = 0; r < n; ++r) {  // nearest smaller position to the left in SA order
        while (!st.empty() && sa[st.back()] > sa[r]) st.pop_back();
        if (!st.empty()) psv[sa[r]] = sa[st.back()];
        st.push_back(r);
    }
    st.clear();
    for (uint32_t r = n; r-- > 0;) {
        while (!st.empty() && sa[st.back()] > sa[r]) st.pop_back();
        if (!st.empty()) nsv[sa[r]] = sa[st.back()];
        st.push_back(r);
    }
    auto lce = [&](uint32_t p, uint32_t q) {
        uint32_t k = 0;
        while (p + k < n && q + k < n && t[p + k] == t[q + k] && t[p + k] >= (uint32_t)ndocs) ++k;
        return k;
    };
    std::vector<uint32_t> lp(n, 0), ln(n, 0);
    for (uint32_t p = 0; p < n; ++p) {
        if (t[p] < (uint32_t)ndocs) continue;
        if (psv[p] != kNo) lp[p] = lce(p, psv[p]);
        if (nsv[p] != kNo) ln[p] = lce(p, nsv[p]);
    }
    auto dist = [&](uint32_t p) { return end[doc_of[p]] - p; };
    // climb to the earliest occurrence of T[p .. p+l)
    uint64_t steps = 0, longest = 0;
    auto earliest = [&](uint32_t p, uint32_t l) {
        uint64_t k = 0;
        for (;; ++k) {
            if (lp[p] >= l) p = psv[p];
            else if (ln[p] >= l) p = nsv[p];
            else break;
        }
        steps += k;
        longest = std::max(longest, k);
        return p;
    };
    std::vector<uint8_t> cand(n, 0);
    std::vector<uint32_t> E(n, kNo);
    std::unordered_map<uint64_t, uint32_t> gmin;
    uint64_t leaves = 0, one_sided = 0, ncand = 0;
    for (int d = 0; d < ndocs; ++d)
        for (uint32_t j = start[d]; j < end[d]; ++j) {
            const uint32_t l = std::max(lp[j], ln[j]);
            if (j + l >= end[d]) break;  // the rest of the doc stays implicit
            ++leaves;
            if (l == 0) continue;
            // side minimum right of sigma.a: nothing smaller on the right inside sigma, the
            // left neighbour in sigma.a; left of it: the right neighbour in sigma.a, nothing
            // smaller on the left inside sigma except terminated copies of sigma (they sort
            // first and are no leaves: implicit doc ends, never branches)
            uint32_t q;
            if (ln[j] < l) q = psv[j];
            else if (lp[j] < l || dist(psv[j]) == l) q = nsv[j];
            else continue;
            ++one_sided;
            const uint32_t e = earliest(q, l);
            E[j] = e;
            if (dist(e) <= l) continue;  // sigma ends E's doc: E's leaf node is sigma's node
            if (dist(q) <= l || t[q + l] != t[e + l]) continue;  // q outside sigma.a
            cand[j] = 1;
            ++ncand;
            const uint64_t key = (uint64_t)e << 20 | l;
            auto it = gmin.find(key);
            if (it == gmin.end()) gmin.emplace(key, j);
            else it->second = std::min(it->second, j);
        }
    Pool pool{pools0, used0};
    uint64_t splits = 0;
    for (int d = 0; d < ndocs; ++d) {
        for (uint32_t j = start[d]; j < end[d]; ++j) {
            const uint32_t l = std::max(lp[j], ln[j]);
            if (j + l >= end[d]) break;
            const bool split = cand[j] && gmin[(uint64_t)E[j] << 20 | l] == j;
            splits += split;
            pool.charge(5);
            if (split) {
                pool.charge(5);
                pool.charge(3);
            }
            pool.charge(3);
        }
        pools_out[d] = pool.pools;
        used_out[d] = pool.used;
    }
    if (stats) {
        stats[0] = leaves;
        stats[1] = splits;
        stats[2] = one_sided;
        stats[3] = steps;
        stats[4] = ncand;
        stats[5] = longest;
    }
    return 0;
}

}  // extern "C"
