// oracle/ref_trace.cpp — TEST INFRASTRUCTURE ONLY (debug build of the reference).
// Interposes the reference's stream-encoder entry point so the per-byte message
// stream that SuffixTree.cpp emits (MSG_COMPRESS / MSG_NO_COMPRESS) can be logged.
// Built with -DPiXiuStr_init_stream=pxref_stream_real applied to PiXiuStr.cpp only.
#include "PiXiuStr.h"
#include <vector>
PiXiuStr *pxref_stream_real(PXSMsg, bool);
static std::vector<int> g_log;
PiXiuStr *PiXiuStr_init_stream(PXSMsg m, bool outside) {
    if (outside) { g_log.push_back(m.chunk_idx_Cmd); g_log.push_back(m.pxs_idx); g_log.push_back(m.val); }
    return pxref_stream_real(m, outside);
}
extern "C" int refx_trace_take(int *out, int cap) {
    int n = (int)g_log.size();
    if (n > cap) return -1;
    for (int i = 0; i < n; ++i) out[i] = g_log[i];
    g_log.clear();
    return n / 3;
}
