// Client code written against the reference's PiXiuCtrl API (README.md:121-150,
// main.cpp:40-75), compiled unchanged against include/PiXiuCtrl.h.
#include <stdio.h>
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
    ctrl.free_prop();
    printf("facade_test: %s (%zu live keys)\n", fails ? "FAILED" : "ok", ref.size());
    return fails ? 1 : 0;
}
