// Host-only parts of the runtime (pixiu_amd/csrc/px_host.h) on the CPU, built by
// tests/test_host_sanitized.py with -fsanitize=address,undefined: the CritBit index
// against std::map (randomized CRUD over keys with escape bytes, iter under prefixes),
// the key maps against std::unordered_map, the block heap over malloc (no two live
// blocks overlap, every byte is returned), and parallel_ranges.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <random>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "px_host.h"
#include "px_route.h"

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            if (++fails > 20) exit(1);                                  \
        }                                                               \
    } while (0)

// the escaped key the CritBit stores (PiXiuStr_init_key: 251 doubled, then 251,0)
static std::string esc_key(const std::string &raw) {
    std::string q;
    for (char c : raw) {
        q.push_back(c);
        if ((uint8_t)c == 251) q.push_back(c);
    }
    q.push_back((char)251);
    q.push_back((char)0);
    return q;
}

static void test_critbit() {
    std::mt19937 rng(19950207);
    // (no byte 251 here: a key whose escaped form first differs from the crit leaf's right
    // after a 251 is not indexed at all -- the reference's `if (!spec_mode) insert()`,
    // CritBitTree.cpp:96-100 -- checked separately below)
    const char alpha[] = {'A', 'B', 'C', (char)250, (char)0, (char)1};
    pxh::CritBit t;
    std::vector<std::string> kp;          // leaf id (chunk) -> stored escaped key
    std::map<std::string, uint32_t> ref;  // escaped key -> live leaf
    std::set<uint32_t> dead;
    auto kpf = [&](const pxh::Leaf &l, uint32_t *len) {
        *len = (uint32_t)kp[l.chunk].size();
        return (const uint8_t *)kp[l.chunk].data();
    };
    for (int op = 0; op < 20000; ++op) {
        std::string raw;
        for (int j = 0, n = 1 + (int)(rng() % 6); j < n; ++j) raw.push_back(alpha[rng() % 6]);
        const std::string q = esc_key(raw);
        const uint32_t r = rng() % 10;
        if (r < 6) {  // setitem
            const uint32_t id = (uint32_t)kp.size();
            kp.push_back(q);
            uint32_t replaced_leaf = ~0u;
            const int rc = t.insert(q, pxh::Leaf{id, 0}, kpf, [&](const pxh::Leaf &l) { replaced_leaf = l.chunk; });
            auto it = ref.find(q);
            CHECK(rc == (it != ref.end() ? 1 : 0));
            if (it != ref.end()) {
                CHECK(replaced_leaf == it->second);
                dead.insert(it->second);
            }
            ref[q] = id;
        } else if (r < 8) {  // delitem
            uint32_t gone = ~0u;
            const int rc = t.remove(q, kpf, [&](const pxh::Leaf &l) { gone = l.chunk; });
            auto it = ref.find(q);
            CHECK(rc == (it != ref.end() ? 0 : 1));
            if (it != ref.end()) {
                CHECK(gone == it->second);
                ref.erase(it);
            }
        } else {  // getitem / contains
            pxh::Leaf l{~0u, 0};
            const bool f = t.lookup(q, kpf, &l);
            auto it = ref.find(q);
            CHECK(f == (it != ref.end()));
            if (f && it != ref.end()) CHECK(l.chunk == it->second);
        }
        if (op % 997 == 0) {  // iter under a one-byte prefix: the live keys under it, in crit-bit
            const std::string p(1, alpha[rng() % 3]);  // order (= byte order of the escaped keys)
            std::vector<pxh::Leaf> got;
            const bool any = t.iter(p, [&](const pxh::Leaf &l) { return kp[l.chunk].compare(0, 1, p) == 0; }, got);
            CHECK(any == !ref.empty());
            std::vector<uint32_t> want;
            for (auto &kv : ref)
                if (kv.first.compare(0, 1, p) == 0) want.push_back(kv.second);
            std::vector<uint32_t> g;
            for (auto &l : got) g.push_back(l.chunk);
            CHECK(g == want);
        }
    }
    size_t live = 0;
    for (auto &kv : ref) live += !dead.count(kv.second);
    CHECK(live == ref.size());
    printf("critbit: %zu live keys, %zu inner nodes\n", ref.size(), t.cbt.size() - t.cbt_free.size());
    // the reference's escape quirk: "A" stored, then "A\xfb" (escaped A 251 251 251 0 against
    // A 251 0: the streams part right after a 251) is neither inserted nor a replace
    pxh::CritBit u;
    kp.assign({esc_key("A"), esc_key("A\xfb"), esc_key("B")});
    CHECK(u.insert(kp[0], pxh::Leaf{0, 0}, kpf, [](const pxh::Leaf &) {}) == 0);
    CHECK(u.insert(kp[1], pxh::Leaf{1, 0}, kpf, [](const pxh::Leaf &) {}) == 2);
    CHECK(u.insert(kp[2], pxh::Leaf{2, 0}, kpf, [](const pxh::Leaf &) {}) == 0);
    pxh::Leaf l{~0u, 0};
    CHECK(u.lookup(kp[0], kpf, &l) && l.chunk == 0);
    CHECK(!u.lookup(kp[1], kpf, nullptr));
    CHECK(u.lookup(kp[2], kpf, &l) && l.chunk == 2);

    // What the runtime's fast paths rely on (px_runtime.cpp resolve_key, the device key
    // index): with clean prefixes (stored prefix = escaped key), every leaf an insert placed
    // (0 or 1) and that no later replace or delete removed is reached by its key's walk --
    // whatever was skipped (2), replaced or deleted since.  Random operations over an
    // alphabet with 251 and 0 (prefix-related keys and skipped inserts everywhere).
    const char alpha2[] = {'a', 'b', (char)251, (char)0};
    for (int trial = 0; trial < 40; ++trial) {
        pxh::CritBit w;
        kp.clear();
        std::map<std::string, uint32_t> placed;  // escaped key -> leaf a walk must reach
        size_t skipped = 0;
        for (int op = 0; op < 600; ++op) {
            std::string raw;
            for (int j = 0, n = 1 + (int)(rng() % 5); j < n; ++j) raw.push_back(alpha2[rng() % 4]);
            const std::string q = esc_key(raw);
            if (rng() % 5 < 4) {
                const uint32_t id = (uint32_t)kp.size();
                kp.push_back(q);
                uint32_t gone = ~0u;
                const int rc = w.insert(q, pxh::Leaf{id, 0}, kpf, [&](const pxh::Leaf &x) { gone = x.chunk; });
                CHECK(rc >= 0 && rc <= 2);
                if (rc == 1) {  // the replaced leaf held the same key
                    CHECK(placed.count(q) && placed[q] == gone);
                }
                if (rc == 2) {
                    ++skipped;
                    CHECK(!w.lookup(q, kpf, nullptr) || placed.count(q));
                } else {
                    placed[q] = id;
                }
            } else {
                uint32_t gone = ~0u;
                if (w.remove(q, kpf, [&](const pxh::Leaf &x) { gone = x.chunk; }) == 0) {
                    CHECK(placed.count(q) && placed[q] == gone);
                    placed.erase(q);
                }
            }
            for (auto &kv : placed) {
                pxh::Leaf f{~0u, 0};
                CHECK(w.lookup(kv.first, kpf, &f) && f.chunk == kv.second);
            }
        }
        if (trial == 0) printf("critbit 251-alphabet: %zu placed keys, %zu skipped inserts\n", placed.size(), skipped);
    }
}

static void test_keymaps() {
    std::mt19937_64 rng(7);
    pxh::PartKeyMap pm;
    pxh::KeyMap km;
    std::unordered_map<std::string, uint32_t> ref;
    for (int i = 0; i < 50000; ++i) {
        std::string k;
        for (int j = 0, n = (int)(rng() % 24); j < n; ++j) k.push_back((char)(rng() % 7 + 250 * (rng() % 2)));
        const uint32_t sh = (uint32_t)(rng() % 1000);
        const auto *kb = (const uint8_t *)k.data();
        auto it = ref.find(k);
        const int64_t prev = km.upsert(kb, k.size(), sh, sh + 1, sh + 2);
        CHECK(prev == (it == ref.end() ? -1 : (int64_t)it->second));
        pm.put(kb, k.size(), sh, sh + 1, sh + 2);
        ref[k] = sh;
        if (i % 5 == 0) {
            uint32_t a, b, c;
            CHECK(pm.find_hint(kb, k.size(), &a, &b, &c) && a == sh && b == sh + 1 && c == sh + 2);
            // the batched form (hash computed by the caller) agrees
            const uint64_t h = pxh::KeyMap::hash(kb, k.size());
            CHECK(pm.slot_addr(h) != nullptr);
            CHECK(pm.find_hint_h(h, kb, k.size(), &a, &b, &c) && a == sh && b == sh + 1 && c == sh + 2);
            std::string miss = k + "\x01\x02\x03";
            CHECK(pm.find((const uint8_t *)miss.data(), miss.size()) == (ref.count(miss) ? (int64_t)ref[miss] : -1));
        }
    }
    CHECK(km.size() == ref.size() && pm.size() == ref.size());
    {  // set_batch's form: one-shot reserve, hash computed by the caller, prefetch address
        pxh::KeyMap m2;
        m2.reserve(ref.size(), 24 * ref.size());
        for (auto &kv : ref) {
            const auto *kb = (const uint8_t *)kv.first.data();
            const uint64_t h = pxh::KeyMap::hash(kb, kv.first.size());
            CHECK(m2.probe_addr(h) != nullptr);
            CHECK(m2.upsert_h(h, kb, kv.first.size(), kv.second, 1, 2) == -1);
            CHECK(m2.upsert_h(h, kb, kv.first.size(), kv.second + 1, 1, 2) == (int64_t)kv.second);
        }
        CHECK(m2.size() == ref.size());
        for (auto &kv : ref) CHECK(m2.find((const uint8_t *)kv.first.data(), kv.first.size()) == kv.second + 1);
    }
    for (auto &kv : ref) {
        CHECK(km.find((const uint8_t *)kv.first.data(), kv.first.size()) == kv.second);
        CHECK(pm.find((const uint8_t *)kv.first.data(), kv.first.size()) == kv.second);
    }
    printf("keymaps: %zu keys\n", ref.size());
}

struct MallocRaw {
    static void *get(uint64_t n) { return malloc(n); }
    static void put(void *p) { free(p); }
};

static void test_heap() {
    std::mt19937 rng(11);
    uint64_t held = 0;
    {
        pxh::BlockHeap<MallocRaw> h(1 << 20);
        struct Blk {
            uint8_t *p;
            uint64_t n;
            uint8_t tag;
        };
        std::vector<Blk> live;
        for (int i = 0; i < 20000; ++i) {
            if (live.empty() || rng() % 3) {
                const uint64_t n = 1 + rng() % (rng() % 8 ? 4096 : 300000);
                auto *p = (uint8_t *)h.alloc(n);
                CHECK(p != nullptr);
                const uint8_t tag = (uint8_t)(i & 0xff);
                memset(p, tag, n);  // (ASan: the whole block is addressable)
                live.push_back(Blk{p, n, tag});
            } else {
                const size_t k = rng() % live.size();
                const Blk b = live[k];
                for (uint64_t j = 0; j < b.n; j += 97) CHECK(b.p[j] == b.tag);  // nobody else wrote here
                CHECK(b.p[b.n - 1] == b.tag);
                h.release(b.p);
                live[k] = live.back();
                live.pop_back();
            }
        }
        // trim with live blocks: only wholly free slabs go back, the live ones stay intact
        const size_t keep_live = std::min<size_t>(live.size(), 40);
        for (size_t k = keep_live; k < live.size(); ++k) h.release(live[k].p);
        live.resize(keep_live);
        const uint64_t peak = h.peak(), before = h.held();
        CHECK(peak >= before);
        h.trim(0);
        CHECK(h.held() <= before && h.held() >= h.live_bytes());
        CHECK(h.peak() == peak);
        for (auto &b : live) {
            for (uint64_t j = 0; j < b.n; j += 97) CHECK(b.p[j] == b.tag);
            h.release(b.p);
        }
        CHECK(h.live_bytes() == 0);
        CHECK(h.cached_free() == h.held());
        held = h.held();
        h.trim(1 << 20);  // keep at most one slab's worth of free bytes
        CHECK(h.held() <= (1u << 20) || h.held() == 0 || h.cached_free() <= (1u << 20));
        h.trim(0);
        CHECK(h.held() == 0);
        auto *p = (uint8_t *)h.alloc(5000);  // and the heap still works afterwards
        CHECK(p != nullptr);
        h.release(p);
    }
    printf("heap: %llu bytes held before trim, all free\n", (unsigned long long)held);
}

static void test_parallel_ranges() {
    for (uint32_t n : {0u, 1u, 2047u, 2048u, 100000u, 1000003u}) {
        std::vector<std::atomic<uint32_t>> hit(n);
        for (auto &x : hit) x.store(0);
        pxh::parallel_ranges(n, 8, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t i = lo; i < hi; ++i) hit[i].fetch_add(1);
        });
        bool once = true;
        for (auto &x : hit) once = once && x.load() == 1;
        CHECK(once);
    }
    printf("parallel_ranges: ok\n");
    for (uint32_t n : {0u, 1u, 65535u, 65536u, 200001u, 1000003u}) {  // parallel_prefix == the serial sum
        std::vector<uint64_t> a(n + 1), b(n + 1, 0);
        auto val = [](uint32_t i) -> uint64_t { return (i * 2654435761u) % 1000u; };
        pxh::parallel_prefix(n, 8, a.data(), val);
        for (uint32_t i = 0; i < n; ++i) b[i + 1] = b[i] + val(i);
        CHECK(a == b);
    }
    printf("parallel_prefix: ok\n");
}

// seg_sort_pairs' pass routing (px_route.h): for 1..8 passes and the callers' aliasings, every
// pass writes buffers it does not read and the last writes the final pair; simulated on host
// arrays the routed passes (stable copies standing in for the scatter) deliver the input intact
static void test_sort_route() {
    int bufk[6], bufv[6];  // distinct addresses: ka, kb, k0, out, out2 ...
    const void *K[6], *V[6];
    for (int i = 0; i < 6; ++i) K[i] = &bufk[i], V[i] = &bufv[i];
    struct Case {
        bool text;
        int kb, out_k, out_v;  // kb: index or -1 (absent); out: indices of the final pair
    };
    // ka = 0, kb = 1, k0 = 2, separate outputs 3 / 4
    const Case cases[] = {
        {true, 1, 1, 4},   // the first suffix sort: kout = kb, vout = sa
        {true, 1, 3, 4},   // separate outputs
        {false, -1, 3, 4}, // the big groups' sort: k0 reused, outputs apart
        {false, -1, 2, 2}, // in place over the input
        {false, 1, 1, 1},  // output = kb
    };
    for (const Case &c : cases) {
        for (uint32_t passes = 1; passes <= px::kRouteMaxPasses; ++passes) {
            const px::BufPair in0 = c.text ? px::BufPair{nullptr, nullptr} : px::BufPair{K[2], V[2]};
            const px::BufPair scratch[4] = {{K[0], V[0]},
                                            {c.kb >= 0 ? K[c.kb] : nullptr, c.kb >= 0 ? V[c.kb] : nullptr},
                                            {c.text ? nullptr : K[2], c.text ? nullptr : V[2]},
                                            {K[c.out_k], V[c.out_v]}};
            const px::BufPair fin{K[c.out_k], V[c.out_v]};
            px::BufPair out[px::kRouteMaxPasses];
            const bool ok = px::sort_route(passes, in0, scratch, fin, out);
            // in place over its input with one scratch pair the passes alternate between two
            // buffers, so only an even count ends in the input: odd counts must be refused
            const bool expect = !(!c.text && c.kb < 0 && px::pair_overlap(in0, fin) && passes % 2 == 1);
            if (ok != expect) fprintf(stderr, "case text=%d kb=%d out=%d/%d passes=%u ok=%d\n", c.text, c.kb, c.out_k, c.out_v, passes, ok);
            CHECK(ok == expect);
            if (!ok) continue;
            CHECK(out[passes - 1].k == fin.k && out[passes - 1].v == fin.v);
            for (uint32_t p = 0; p < passes; ++p) {
                const px::BufPair in = p == 0 ? in0 : out[p - 1];
                CHECK(!px::pair_overlap(out[p], in));
                CHECK(out[p].k && out[p].v);
            }
            // the data survives the chain (every buffer holds the label of the pass that wrote it)
            int val = 100;
            for (int i = 0; i < 6; ++i) bufk[i] = bufv[i] = -1;
            if (!c.text) bufk[2] = bufv[2] = val;
            for (uint32_t p = 0; p < passes; ++p) {
                const px::BufPair in = p == 0 ? in0 : out[p - 1];
                const int ink = in.k ? *(const int *)in.k : val, inv = in.v ? *(const int *)in.v : val;
                CHECK(ink == val && inv == val);
                *(int *)out[p].k = val + 1;
                *(int *)out[p].v = val + 1;
                ++val;
            }
            CHECK(*(const int *)fin.k == val && *(const int *)fin.v == val);
        }
    }
    // the parity routing that faulted: 7 and 5 passes from the text with kout == kb
    for (uint32_t passes : {5u, 7u}) {
        const px::BufPair scratch[4] = {{K[0], V[0]}, {K[1], V[1]}, {nullptr, nullptr}, {K[1], V[4]}};
        px::BufPair out[px::kRouteMaxPasses];
        CHECK(px::sort_route(passes, px::BufPair{nullptr, nullptr}, scratch, px::BufPair{K[1], V[4]}, out));
        CHECK(out[passes - 2].k == K[0]);  // the pass before the last must not write kb
    }
    CHECK(!px::sort_route(0, px::BufPair{nullptr, nullptr}, nullptr, px::BufPair{K[0], V[0]}, nullptr));
    CHECK(!px::sort_route(9, px::BufPair{nullptr, nullptr}, nullptr, px::BufPair{K[0], V[0]}, nullptr));
    printf("sort_route: ok\n");
}

int main() {
    test_sort_route();
    test_critbit();
    test_keymaps();
    test_heap();
    test_parallel_ranges();
    printf("host_test: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
