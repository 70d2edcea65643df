// Client code written against the reference's PiXiuCtrl API (README.md:121-150,
// main.cpp:40-75), compiled unchanged against include/PiXiuCtrl.h.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <vector>
#include <string>

#include "PiXiuCtrl.h"

static int fails = 0;
#define CHECK(c)                                                    \
    do {                                                            \
        if (!(c)) {                                                 \
            fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                \
        }                                                           \
    } while (0)

int main() {
    PiXiuCtrl ctrl;
    ctrl.init_prop();
    // README example
    std::string key = "WhoAmI", val = "ChengLin";
    ctrl.setitem((uint8_t *)key.c_str(), (int)key.size(), (uint8_t *)val.c_str(), (int)val.size());
    CHECK(ctrl.contains((uint8_t *)key.c_str(), (int)key.size()));
    PXSGen *gen = ctrl.getitem((uint8_t *)key.c_str(), (int)key.size());
    CHECK(gen != NULL);
    std::string got;
    uint8_t rv;
    while (gen->operator()(rv)) got.push_back((char)rv);
    PXSGen_free(gen);
    CHECK(got == std::string("WhoAmI\xfb\x00", 8) + "ChengLin\xfb\x02");
    CHECK(ctrl.delitem((uint8_t *)key.c_str(), (int)key.size()) == 0);
    CHECK(!ctrl.contains((uint8_t *)key.c_str(), (int)key.size()));
    CHECK(ctrl.getitem((uint8_t *)key.c_str(), (int)key.size()) == NULL);
    ctrl.free_prop();

    // CLI transcript (README.md:71-95): saved bytes = len(cmd) - compressed len (main.cpp:67)
    ctrl.init_prop();
    const char *cmds[] = {"SET 123::321", "SET BOBO::https://www.zhihu.com/question/55439090",
                          "SET BOBO1::https://www.zhihu.com/question/22454692"};
    int saved[3];
    for (int i = 0; i < 3; ++i) {
        std::string cmd = cmds[i];
        size_t pos = cmd.find("::");
        std::string k = cmd.substr(4, pos - 4), v = cmd.substr(pos);
        ctrl.setitem((uint8_t *)k.c_str(), (int)k.size(), (uint8_t *)v.c_str(), (int)v.size());
        saved[i] = (int)cmd.size() - ctrl.st.cbt_chunk->getitem(ctrl.st.local_chunk.used_num - 1)->len;
    }
    CHECK(saved[0] == 0 && saved[1] == 0 && saved[2] == 27);
    char *repr = ctrl.getitem((uint8_t *)"BOBO1", 5)->consume_repr();
    CHECK(strcmp(repr, "BOBO1::https://www.zhihu.com/question/22454692") == 0);
    free(repr);

    // randomized CRUD vs std::map (PiXiuCtrl.cpp:176-226 shape)
    std::map<std::string, std::string> ref;
    unsigned s = 12345;
    auto rnd = [&]() { return (s = s * 1103515245u + 12345u) >> 8; };
    for (int i = 0; i < 400; ++i) {
        std::string k, v;
        for (int j = 0, n = 1 + rnd() % 5; j < n; ++j) k += "ABCDE"[rnd() % 5];
        for (int j = 0, n = 1 + rnd() % 40; j < n; ++j) v += "ABCDE"[rnd() % 5];
        int r = ctrl.setitem((uint8_t *)k.c_str(), (int)k.size(), (uint8_t *)v.c_str(), (int)v.size());
        CHECK(r == (ref.count(k) ? CBT_SET_REPLACE : 0));
        ref[k] = v;
        if (rnd() % 3 == 0) {
            auto it = ref.begin();
            std::advance(it, rnd() % ref.size());
            std::string d = it->first;
            CHECK(ctrl.delitem((uint8_t *)d.c_str(), (int)d.size()) == 0);
            ref.erase(d);
        }
    }
    for (auto &kv : ref) {
        char *r = ctrl.getitem((uint8_t *)kv.first.c_str(), (int)kv.first.size())->consume_repr();
        CHECK(std::string(r) == kv.first + kv.second);
        free(r);
    }
    // iter (PiXiuCtrl.cpp:71-75): records under a prefix in crit-bit order, i.e. in the
    // order of their escaped keys incl. the 251,0 terminator; nothing for an absent prefix
    const std::string term("\xfb\x00", 2);
    std::vector<std::string> want;
    for (auto &kv : ref)
        if (kv.first[0] == 'A') want.push_back(kv.first);
    std::sort(want.begin(), want.end(), [&](const std::string &a, const std::string &b) { return a + term < b + term; });
    CBTGen *it = ctrl.iter((uint8_t *)"A", 1);
    CHECK(it != NULL);
    size_t got_n = 0;
    PXSGen *g = NULL;
    while (it && (*it)(g)) {
        char *r = g->consume_repr();
        CHECK(got_n < want.size() && std::string(r) == want[got_n] + ref[want[got_n]]);
        free(r);
        ++got_n;
    }
    CHECK(got_n == want.size() && got_n > 0);
    CBTGen_free(it);
    it = ctrl.iter((uint8_t *)"F", 1);
    CHECK(it != NULL && !(*it)(g));
    CBTGen_free(it);
    ctrl.free_prop();
    ctrl.init_prop();
    CHECK(ctrl.iter((uint8_t *)"A", 1) == NULL);  // empty tree: NULL generator

    // a slot-full chunk compacted by a direct reinsert (PiXiuCtrl.cpp:88-114), and an iter
    // across many expansion windows.  The records go in through the C ABI in one batch
    // (65,545 single-record setitems would each run the whole GPU pipeline).
    {
        const int n = PXC_STR_NUM + 10;
        std::vector<std::string> ks(n), vs(n);
        std::string kb, vb;
        std::vector<uint64_t> ko(1, 0), vo(1, 0);
        for (int i = 0; i < n; ++i) {
            char b[16];
            snprintf(b, sizeof b, "r%06d", i);
            ks[i] = b;
            vs[i] = std::string("v") + std::to_string(i * 7919 % 100003);
            kb += ks[i];
            vb += vs[i];
            ko.push_back(kb.size());
            vo.push_back(vb.size());
        }
        CHECK(px_set_batch(ctrl.ctx, n, (const uint8_t *)kb.data(), ko.data(), (const uint8_t *)vb.data(), vo.data(), 0,
                           NULL) == PX_OK);
        std::vector<bool> live(n, true);
        for (int i = 0; i < PXC_STR_NUM; i += 7) {  // 15 % of chunk 0: no trigger fires
            CHECK(ctrl.delitem((uint8_t *)ks[i].c_str(), (int)ks[i].size()) == 0);
            live[i] = false;
        }
        PiXiuChunk *c0 = ctrl.chunk_at(0);
        ctrl.reinsert(c0);
        CHECK(c0 == NULL);
        PiXiuChunk *live_chunk = ctrl.chunk_at(1);  // (the records went in through the C ABI)
        ctrl.reinsert(live_chunk);                  // the live chunk is not compacted
        CHECK(live_chunk != NULL);
        PiXiuChunk *again = ctrl.chunk_at(0);  // nor a chunk with nothing live left
        ctrl.reinsert(again);
        CHECK(again != NULL);
        for (int i = 0; i < n; i += 13) {
            PXSGen *gi = ctrl.getitem((uint8_t *)ks[i].c_str(), (int)ks[i].size());
            CHECK((gi != NULL) == live[i]);
            if (!gi) continue;
            char *r = gi->consume_repr();
            CHECK(std::string(r) == ks[i] + vs[i]);
            free(r);
        }
        // every live record left chunk 0; iter walks them all in key order, 64 per window
        uint32_t m = 0;
        std::vector<px_rec> recs(n);
        CHECK(px_iter(ctrl.ctx, (const uint8_t *)"r", 1, recs.data(), (uint32_t)recs.size(), &m) == PX_OK);
        size_t nlive = 0;
        for (int i = 0; i < n; ++i) nlive += live[i];
        CHECK(m == nlive);
        bool moved = true;
        for (uint32_t j = 0; j < m; ++j) moved = moved && recs[j].chunk > 0;
        CHECK(moved);
        CBTGen *ig = ctrl.iter((uint8_t *)"r00", 3);
        size_t seen = 0, want_n = 0;
        std::vector<std::string> want_k;
        for (int i = 0; i < 10000; ++i)
            if (live[i]) want_k.push_back(ks[i]);
        PXSGen *x = NULL;
        while (ig && (*ig)(x)) {
            char *r = x->consume_repr();
            CHECK(seen < want_k.size() && std::string(r) == want_k[seen] + vs[atoi(want_k[seen].c_str() + 1)]);
            free(r);
            ++seen;
        }
        want_n = want_k.size();
        CHECK(seen == want_n && want_n > 3 * CBTGen::kIterWindow);
        CBTGen_free(ig);
    }
    ctrl.free_prop();

    // write-behind setitem: 3,000 one-record calls with repeated keys return what the
    // reference returns at once, and store the same bytes in the same slots as a context
    // without the queue fed the same calls
    {
        ctrl.init_prop();
        px_opts o;
        memset(&o, 0, sizeof o);
        px_ctx *plain = px_open(&o);  // defer_bytes = 0
        std::map<std::string, int> seen;
        std::vector<std::string> ks;
        unsigned t = 777;
        auto rn = [&]() { return (t = t * 1103515245u + 12345u) >> 8; };
        for (int i = 0; i < 3000; ++i) {
            char b[32];
            snprintf(b, sizeof b, "http://q/%05u", rn() % 2500);
            std::string k = b, v = "::";
            for (int j = 0, n = 20 + rn() % 200; j < n; ++j) v += "abcdefgh<>/="[rn() % 12];
            const int r = ctrl.setitem((uint8_t *)k.c_str(), (int)k.size(), (uint8_t *)v.c_str(), (int)v.size());
            CHECK(r == (seen.count(k) ? CBT_SET_REPLACE : 0));
            uint64_t ko[2] = {0, k.size()}, vo[2] = {0, v.size()};
            px_set_result pr;
            CHECK(px_set_batch(plain, 1, (const uint8_t *)k.data(), ko, (const uint8_t *)v.data(), vo, 0, &pr) == PX_OK);
            CHECK((int)pr.replaced == r && pr.chunk != PX_PENDING);
            seen[k] = 1;
            ks.push_back(k);
        }
        px_stats sd, sp;
        CHECK(px_stats_get(ctrl.ctx, &sd) == PX_OK && px_stats_get(plain, &sp) == PX_OK);
        CHECK(sd.deferred_records == 3000 && sd.deferred_flushes >= 1 && sd.deferred_mismatch == 0);
        CHECK(sd.records == sp.records && sd.comp_bytes == sp.comp_bytes && sd.chunks == sp.chunks);
        bool same = true;
        for (size_t i = 0; i < ks.size(); i += 7) {
            uint64_t ko[2] = {0, ks[i].size()};
            px_rec ra, rb;
            uint32_t sa = 0, sb = 0;
            px_locate_batch(ctrl.ctx, 1, (const uint8_t *)ks[i].data(), ko, &ra, &sa);
            px_locate_batch(plain, 1, (const uint8_t *)ks[i].data(), ko, &rb, &sb);
            same = same && sa == PX_OK && sb == PX_OK && ra.chunk == rb.chunk && ra.idx == rb.idx;
            std::vector<uint8_t> ba(70000), bb(70000);
            uint64_t oa[2], ob[2];
            px_export(ctrl.ctx, 1, &ra, ba.data(), ba.size(), oa);
            px_export(plain, 1, &rb, bb.data(), bb.size(), ob);
            same = same && oa[1] == ob[1] && memcmp(ba.data(), bb.data(), oa[1]) == 0;
        }
        CHECK(same);
        // the CLI's chunk view after one more queued call (main.cpp:67)
        std::string k = "BOBO1", v = "::https://www.zhihu.com/question/22454692";
        ctrl.setitem((uint8_t *)k.c_str(), 5, (uint8_t *)v.c_str(), (int)v.size());
        PiXiuStr *last = ctrl.st.cbt_chunk->getitem(ctrl.st.local_chunk.used_num - 1);
        CHECK(last != NULL && last->len > 0);
        px_close(plain);

        // a ready doc (setitem(doc, 0, NULL, 0, reinsert), PiXiuCtrl.cpp:39-40): stored as it is
        std::string doc = std::string("RAWKEY\xfb\x00", 8) + "raw value bytes" + std::string("\xfb\x02", 2);
        std::vector<uint8_t> pxs(2 + doc.size());
        const uint16_t dl = (uint16_t)doc.size();
        memcpy(pxs.data(), &dl, 2);
        memcpy(pxs.data() + 2, doc.data(), doc.size());
        CHECK(ctrl.setitem(pxs.data(), 0, NULL, 0, true) == 0);
        CHECK(ctrl.setitem(pxs.data(), 0, NULL, 0, false) == CBT_SET_REPLACE);
        PXSGen *rg = ctrl.getitem((uint8_t *)"RAWKEY", 6);
        CHECK(rg != NULL);
        std::string rgot;
        uint8_t c;
        while (rg && (*rg)(c)) rgot.push_back((char)c);
        PXSGen_free(rg);
        CHECK(rgot == doc);
        CHECK(ctrl.setitem(NULL, 0, (uint8_t *)"x", 1) < 0);  // (the reference asserts k_len)

        // a queued record whose store fails is reported, not lost silently (PX_DEBUG_SET_THROW:
        // the batch throws bad_alloc inside the flush a read triggers)
        CHECK(ctrl.setitem((uint8_t *)"FAILKEY", 7, (uint8_t *)"v", 1) == 0);
        setenv("PX_TEST_HOOKS", "1", 1);  // (arms the runtime's fault-injecting hooks)
        setenv("PX_DEBUG_SET_THROW", "1", 1);
        CHECK(!ctrl.contains((uint8_t *)"FAILKEY", 7));
        unsetenv("PX_DEBUG_SET_THROW");
        CHECK(ctrl.flush() == PX_ENOMEM);
        CHECK(ctrl.flush() == PX_OK);
        CHECK(ctrl.setitem((uint8_t *)"FAILKEY", 7, (uint8_t *)"v", 1) == 0);
        CHECK(ctrl.flush() == PX_OK && ctrl.contains((uint8_t *)"FAILKEY", 7));

        // the failure surfacing inside sync_pending (a live-chunk read), then a setitem: the new
        // record is kept (queued) and the earlier failure is returned in its place, once
        CHECK(ctrl.setitem((uint8_t *)"LOSTKEY", 7, (uint8_t *)"w", 1) == 0);
        setenv("PX_DEBUG_SET_THROW", "1", 1);
        const uint16_t un = ctrl.st.local_chunk.used_num;  // (sync_pending: the flush throws)
        (void)un;
        unsetenv("PX_DEBUG_SET_THROW");
        CHECK(ctrl.setitem((uint8_t *)"NEXTKEY", 7, (uint8_t *)"x", 1) == -PX_ENOMEM);
        CHECK(ctrl.flush() == PX_OK);
        CHECK(ctrl.flush() == PX_OK);
        CHECK(ctrl.contains((uint8_t *)"NEXTKEY", 7) && !ctrl.contains((uint8_t *)"LOSTKEY", 7));
        PiXiuStr *nl = ctrl.st.cbt_chunk->getitem(ctrl.st.local_chunk.used_num - 1);
        CHECK(nl != NULL && nl->len > 0);

        // a generator that outlives free_prop yields nothing and says why
        PXSGen *late = ctrl.getitem((uint8_t *)"RAWKEY", 6);
        CHECK(late != NULL);
        ctrl.free_prop();
        CHECK(late && !(*late)(c) && late->status == PX_EINVAL);
        PXSGen_free(late);
    }
    printf("facade_test: %s (%zu live keys)\n", fails ? "FAILED" : "ok", ref.size());
    return fails ? 1 : 0;
}
