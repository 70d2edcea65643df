// tools/proto/lpf_proto.cpp — TEST/DESIGN PROTOTYPE ONLY (never linked into the product).
//
// CPU restatement of the parallel reformulation of the GST walk: the
// encoder message stream of one shard computed from a suffix array instead of an
// online Ukkonen walk.  For byte i of doc `cur`:
//   L(i)   = length of the longest suffix of cur[0..i] that occurs earlier in the shard
//            text (an earlier doc, or cur at an earlier start);  L(-1) = 0 per doc
//   C(i)   = COMPRESS iff L(i) == L(i-1) + 1, else PASS
//   msg(i) = (doc, pos) of the earliest occurrence E of cur[i-L(i)+1 .. i]: pos = E + L(i) - 1
// (The edge label the reference reads is the first leaf created under the active
// point, SuffixTree.cpp:154-157,211-217, i.e. the earliest occurrence.)  A conservative
// check flags shards where the reference's stale (act_chunk_idx, act_direct) pair could
// matter (SuffixTree.cpp:171,184 vs 232-249): every PASS step with L(i) >= 1 must keep
// the earliest occurrence's doc.
//
// extern "C" lpf_messages(): docs in CSR -> one u32 message per doc byte
// (idx << 16 | pos, or 0xffffffff for PASS) + flags.  Test infrastructure compares it
// with the oracle.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Sa {
    std::vector<uint32_t> sa, isa, lcp;  // lcp[r] = lcp(sa[r-1], sa[r])
};

// prefix doubling (std::sort), symbols: bytes, then unique separators
Sa build_sa(const std::vector<uint32_t> &t, uint64_t *active_log) {
    const uint32_t n = (uint32_t)t.size();
    Sa s;
    s.sa.resize(n);
    s.isa.resize(n);
    std::vector<uint32_t> rank(t), tmp(n);
    for (uint32_t i = 0; i < n; ++i) s.sa[i] = i;
    for (uint32_t h = 1;; h <<= 1) {
        auto key = [&](uint32_t i) { return std::make_pair(rank[i], i + h < n ? rank[i + h] + 1 : 0u); };
        std::sort(s.sa.begin(), s.sa.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
        tmp[s.sa[0]] = 0;
        uint32_t groups_open = 0;
        for (uint32_t r = 1; r < n; ++r) {
            bool same = key(s.sa[r - 1]) == key(s.sa[r]);
            tmp[s.sa[r]] = tmp[s.sa[r - 1]] + (same ? 0 : 1);
            groups_open += same;
        }
        rank = tmp;
        if (active_log) active_log[__builtin_ctz(h)] = groups_open;
        if (tmp[s.sa[n - 1]] == n - 1) break;
    }
    for (uint32_t r = 0; r < n; ++r) s.isa[s.sa[r]] = r;
    // Kasai
    s.lcp.assign(n, 0);
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (s.isa[i] == 0) {
            k = 0;
            continue;
        }
        uint32_t j = s.sa[s.isa[i] - 1];
        while (i + k < n && j + k < n && t[i + k] == t[j + k]) ++k;
        s.lcp[s.isa[i]] = k;
        if (k) --k;
    }
    return s;
}

struct Rmq {  // sparse table, min
    std::vector<std::vector<uint32_t>> t;
    void build(const std::vector<uint32_t> &a) {
        t.assign(1, a);
        for (uint32_t k = 1; (1u << k) <= a.size(); ++k) {
            const auto &p = t[k - 1];
            std::vector<uint32_t> c(a.size() - (1u << k) + 1);
            for (size_t i = 0; i < c.size(); ++i) c[i] = std::min(p[i], p[i + (1u << (k - 1))]);
            t.push_back(std::move(c));
        }
    }
    uint32_t q(uint32_t l, uint32_t r) const {  // min a[l..r], l <= r
        uint32_t k = 31 - __builtin_clz(r - l + 1);
        return std::min(t[k][l], t[k][r - (1u << k) + 1]);
    }
};

}  // namespace

extern "C" {

// docs: CSR bytes.  msg: one u32 per doc byte (same CSR offsets).  Returns the number
// of PASS steps that fail the stale-pair check (0: the message stream is the
// reference's); stats[0..31] = open suffix groups after each doubling step.
long lpf_messages(int ndocs, const uint8_t *docs, const uint64_t *off, uint32_t *msg, uint64_t *stats) {
    std::vector<uint32_t> t;
    std::vector<uint32_t> doc_of, start_of(ndocs);
    for (int d = 0; d < ndocs; ++d) {
        start_of[d] = (uint32_t)t.size();
        for (uint64_t p = off[d]; p < off[d + 1]; ++p) {
            t.push_back(docs[p]);
            doc_of.push_back((uint32_t)d);
        }
        t.push_back(256u + (uint32_t)d);  // unique separator: no match crosses a doc end
        doc_of.push_back((uint32_t)d);
    }
    const uint32_t n = (uint32_t)t.size();
    Sa s = build_sa(t, stats);
    Rmq lcp_min, pos_min;
    lcp_min.build(s.lcp);
    pos_min.build(s.sa);
    // lpf(p): longest prefix of suffix p occurring at an earlier start (nearest ranks with a
    // smaller position on either side; lcp between ranks is the lcp-array minimum)
    std::vector<uint32_t> lpf(n, 0), st;
    for (int dir = 0; dir < 2; ++dir) {
        st.clear();
        for (uint32_t k = 0; k < n; ++k) {
            uint32_t r = dir == 0 ? k : n - 1 - k;
            uint32_t p = s.sa[r];
            while (!st.empty() && s.sa[st.back()] > p) st.pop_back();
            if (!st.empty()) {
                uint32_t r2 = st.back();
                uint32_t l = dir == 0 ? lcp_min.q(r2 + 1, r) : lcp_min.q(r + 1, r2);
                lpf[p] = std::max(lpf[p], l);
            }
            st.push_back(r);
        }
    }
    long flagged = 0;
    for (int d = 0; d < ndocs; ++d) {
        const uint32_t b = start_of[d], e = b + (uint32_t)(off[d + 1] - off[d]);
        uint32_t js = b;  // start of the longest earlier-occurring suffix
        int64_t prevL = 0;
        int64_t prev_doc = -1;
        for (uint32_t i = b; i < e; ++i) {
            while (js <= i && js + lpf[js] <= i) ++js;
            const int64_t L = (int64_t)i - js + 1;
            const bool comp = L == prevL + 1;
            int64_t edoc = -1;
            uint32_t m = 0xffffffffu;
            if (L > 0) {
                // SA interval of suffixes sharing >= L symbols with suffix js, then its min position
                const uint32_t r = s.isa[js];
                uint32_t lo = r, hi = r;
                {
                    uint32_t a = 0, z = r;  // smallest lo with min lcp[lo+1..r] >= L
                    while (a < z) {
                        uint32_t mid = (a + z) / 2;
                        if (lcp_min.q(mid + 1, r) >= (uint32_t)L) z = mid; else a = mid + 1;
                    }
                    lo = a;
                    a = r;
                    z = n - 1;  // largest hi with min lcp[r+1..hi] >= L
                    while (a < z) {
                        uint32_t mid = (a + z + 1) / 2;
                        if (lcp_min.q(r + 1, mid) >= (uint32_t)L) a = mid; else z = mid - 1;
                    }
                    hi = a;
                }
                const uint32_t E = pos_min.q(lo, hi);
                edoc = doc_of[E];
                if (comp) m = (uint32_t)edoc << 16 | (uint32_t)(E - start_of[edoc] + L - 1);
            }
            // stale-pair check: a PASS step can leave the reference's (act_chunk_idx,
            // act_direct) stale only if its split loop ends inside an edge (not at a node,
            // SuffixTree.cpp:280-283), i.e. alpha' = cur[i-L+1 .. i-1] is implicit.  With
            // s = cur[i-L .. i-1] (which occurs earlier, L <= L(i-1)): if s's earliest
            // occurrence is followed by a byte y (y != c), alpha' has two extensions and is
            // a node.  So only steps whose s has its earliest occurrence at a doc end are flagged.
            if (!comp && L >= 2) {
                const uint32_t j = i - (uint32_t)L;
                const uint32_t r = s.isa[j];
                uint32_t a = 0, z = r;
                while (a < z) {
                    uint32_t mid = (a + z) / 2;
                    if (lcp_min.q(mid + 1, r) >= (uint32_t)L) z = mid; else a = mid + 1;
                }
                const uint32_t lo = a;
                a = r;
                z = n - 1;
                while (a < z) {
                    uint32_t mid = (a + z + 1) / 2;
                    if (lcp_min.q(r + 1, mid) >= (uint32_t)L) a = mid; else z = mid - 1;
                }
                const uint32_t Es = pos_min.q(lo, a);
                if (t[Es + L] >= 256u) ++flagged;  // followed by its doc's separator
            }
            (void)prev_doc;
            msg[off[d] + (i - b)] = m;
            prevL = L;
            prev_doc = edoc;
        }
    }
    // the same stream from lpf alone (the GPU formulation): C(i) = lpf(i) >= 1
    // unless i = reach(J-1) = J-1+lpf(J-1) for a J whose range is non-empty (lpf(J) >=
    // lpf(J-1)); a run of lpf(J) - lpf(J-1) >= 7 COMPRESS steps ends at b = J+lpf(J)-1 with
    // the earliest occurrence of T[J..J+lpf(J)) (and of one byte less at b-1 if T[b] is 251)
    long alt_diff = 0;
    for (int d = 0; d < ndocs; ++d) {
        const uint32_t b0 = start_of[d], e = b0 + (uint32_t)(off[d + 1] - off[d]);
        std::vector<uint32_t> m2(e - b0);
        for (uint32_t i = b0; i < e; ++i) m2[i - b0] = lpf[i] >= 1 ? 0u : 0xffffffffu;
        auto E = [&](uint32_t J, uint32_t l) {
            const uint32_t r = s.isa[J];
            uint32_t a = 0, z = r;
            while (a < z) { uint32_t mid = (a + z) / 2; if (lcp_min.q(mid + 1, r) >= l) z = mid; else a = mid + 1; }
            const uint32_t lo = a;
            a = r; z = n - 1;
            while (a < z) { uint32_t mid = (a + z + 1) / 2; if (lcp_min.q(r + 1, mid) >= l) a = mid; else z = mid - 1; }
            const uint32_t Ep = pos_min.q(lo, a);
            return (uint32_t)doc_of[Ep] << 16 | (Ep - start_of[doc_of[Ep]] + l - 1);
        };
        for (uint32_t J = b0; J < e; ++J) {
            const uint32_t lp = J > b0 ? lpf[J - 1] : 0;
            if (J > b0 && lpf[J] + 0 >= lp && J - 1 + lp < e) m2[J - 1 + lp - b0] = 0xffffffffu;
        }
        for (uint32_t J = b0; J < e; ++J) {
            const uint32_t lp = J > b0 ? lpf[J - 1] : 0;
            if (lpf[J] >= lp + 7) {
                const uint32_t b = J + lpf[J] - 1;
                m2[b - b0] = E(J, lpf[J]);
                if (t[b] == 251) m2[b - 1 - b0] = E(J, lpf[J] - 1);
            }
        }
        for (uint32_t i = b0; i < e; ++i) {
            const uint32_t a = msg[off[d] + (i - b0)], b = m2[i - b0];
            if ((a == 0xffffffffu) != (b == 0xffffffffu)) ++alt_diff;
        }
        if (stats) stats[31] += alt_diff;
        // the GPU formulation's stream replaces the scan's (tokens only use run ends)
        for (uint32_t i = b0; i < e; ++i) msg[off[d] + (i - b0)] = m2[i - b0];
    }
    return flagged;
}

}  // extern "C"
