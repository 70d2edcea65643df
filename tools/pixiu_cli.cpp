// pixiu_cli — the reference's REPL (main.cpp:40-75 behaviour) on the GPU core:
//   GET <key>        print the visible bytes of the stored doc
//   SET <key>::<v>   store, print bytes saved (len(command) - compressed length)
//   ~                quit
#include <iostream>
#include <string>

#include "PiXiuCtrl.h"

int main() {
    PiXiuCtrl ctrl;
    ctrl.init_prop();
    std::string cmd;
    long total = 0;
    while (std::cout << "Command: " && std::getline(std::cin, cmd)) {
        if (!cmd.empty() && cmd[0] == '~') break;
        if (cmd.rfind("GET ", 0) == 0) {
            PXSGen *g = ctrl.getitem((uint8_t *)cmd.c_str() + 4, (int)cmd.size() - 4);
            if (g) {
                char *s = g->consume_repr();
                std::cout << s << std::endl;
                free(s);
            }
        } else if (cmd.rfind("SET ", 0) == 0) {
            size_t pos = cmd.find("::");
            if (pos == std::string::npos) continue;
            std::string k = cmd.substr(4, pos - 4), v = cmd.substr(pos);
            ctrl.setitem((uint8_t *)k.c_str(), (int)k.size(), (uint8_t *)v.c_str(), (int)v.size());
            int diff = (int)cmd.size() - ctrl.st.cbt_chunk->getitem(ctrl.st.local_chunk.used_num - 1)->len;
            total += diff;
            std::cout << "saved " << diff << "\ntotal saved " << total << std::endl;
        }
    }
    ctrl.free_prop();
    return 0;
}
