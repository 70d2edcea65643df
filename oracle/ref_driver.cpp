// oracle/ref_driver.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// A thin extern "C" driver around the *unmodified* reference sources, which are
// compiled by path from /root/reference/src by oracle/Makefile into
// oracle/_ref/libpxref.so.  Nothing from the reference is copied here: this file
// only calls the reference's public surface (PiXiuCtrl.h:7-26, PiXiuStr.h:61-100)
// so that tests/ and tools/make_golden.py can (a) pin the clean-room restatement
// oracle/pxo.cpp against the real thing and (b) emit golden vectors into
// tests/golden/.  The reference keeps process-global state (PiXiuStr.cpp:4,17-26;
// SuffixTree.cpp:5-6), so exactly one controller lives in this library.
#include "PiXiuCtrl.h"

#include <stdint.h>
#include <string.h>

#include <vector>

static PiXiuCtrl g_ctrl;
static PiXiuChunk *g_last_chunk = nullptr;
static uint32_t g_chunk_serial = 0;
static bool g_live = false;
static std::vector<PiXiuChunk *> g_chunks;  // chunk by serial (nullptr once reinserted)

extern "C" {

void refx_init(void) {
    if (g_live) { g_ctrl.free_prop(); }
    g_ctrl.init_prop();                      // PiXiuCtrl.cpp:77-81
    g_last_chunk = g_ctrl.st.cbt_chunk;
    g_chunk_serial = 0;
    g_chunks.assign(1, g_last_chunk);
    g_live = true;
}

void refx_free(void) {
    if (g_live) { g_ctrl.free_prop(); }     // PiXiuCtrl.cpp:83-86
    g_live = false;
}

// PiXiuCtrl::setitem (PiXiuCtrl.cpp:12-47).  Reports which chunk (0-based
// rotation count) and which chunk-local slot the record landed in.
int refx_setitem(const uint8_t *k, int klen, const uint8_t *v, int vlen,
                 uint32_t *chunk_no, uint32_t *idx) {
    int rc = g_ctrl.setitem((uint8_t *)k, klen, (uint8_t *)v, vlen);
    if (g_ctrl.st.cbt_chunk != g_last_chunk) {
        g_last_chunk = g_ctrl.st.cbt_chunk;
        g_chunk_serial++;
        g_chunks.push_back(g_last_chunk);
    }
    if (chunk_no) *chunk_no = g_chunk_serial;
    if (idx) *idx = (uint32_t)(g_ctrl.st.local_chunk.used_num - 1);
    return rc;
}

// Compressed bytes of the record stored by the last setitem (main.cpp:67 path).
int refx_last_comp(uint8_t *out, int cap) {
    PiXiuStr *p = g_ctrl.st.cbt_chunk->getitem(g_ctrl.st.local_chunk.used_num - 1);
    int n = p->len;
    if (n > cap) return -1;
    memcpy(out, p->data, (size_t)n);
    return n;
}

// Drain a generator into out; returns bytes produced, -2 if more than cap.
static int drain(PXSGen *gen, uint8_t *out, int cap) {
    uint8_t rv;
    int n = 0;
    while (gen->operator()(rv)) {
        if (n >= cap) { PXSGen_free(gen); return -2; }
        out[n++] = rv;
    }
    PXSGen_free(gen);
    return n;
}

// PiXiuCtrl::getitem (PiXiuCtrl.cpp:59-61) -> PXSGen drained. -1 == NULL.
int refx_getitem(const uint8_t *k, int klen, uint8_t *out, int cap) {
    PXSGen *gen = g_ctrl.getitem((uint8_t *)k, klen);
    if (gen == nullptr) return -1;
    return drain(gen, out, cap);
}

// PiXiuCtrl::reinsert(PiXiuChunk *&) (PiXiuCtrl.cpp:88-114) called directly on the chunk
// with the given serial; -1 for the live chunk or one already freed
int refx_reinsert(uint32_t serial) {
    if (serial >= g_chunks.size() || !g_chunks[serial] || g_chunks[serial] == g_ctrl.st.cbt_chunk) return -1;
    g_ctrl.reinsert(g_chunks[serial]);  // (sets the entry to NULL, as the reference's reference argument)
    if (g_ctrl.st.cbt_chunk != g_last_chunk) {  // the re-sets rotated the live chunk
        g_last_chunk = g_ctrl.st.cbt_chunk;
        g_chunk_serial++;
        g_chunks.push_back(g_last_chunk);
    }
    return 0;
}

int refx_contains(const uint8_t *k, int klen) {
    return g_ctrl.contains((uint8_t *)k, klen) ? 1 : 0;
}

int refx_delitem(const uint8_t *k, int klen) {
    return g_ctrl.delitem((uint8_t *)k, klen);
}

// CritBitTree::getitem's lookup (CritBitTree.cpp:185-195) stopped before the parse: the
// located record's slot and compressed bytes; -5 when the key is absent.
int refx_locate(const uint8_t *k, int klen, uint8_t *out, int cap, uint32_t *idx) {
    if (g_ctrl.cbt.root == NULL) return -5;
    PiXiuStr *src = PiXiuStr_init_key((uint8_t *)k, klen);
    auto ret = g_ctrl.cbt.find_best_match(src);
    auto pa = (CBTInner *)ret.pa;
    auto chunk = (PiXiuChunk *)ret.crit_node;
    int ci = pa == NULL ? g_ctrl.cbt.chunk_idx : pa->chunk_idx_arr[ret.pa_direct];
    PiXiuStr *p = chunk->getitem(ci);
    bool eq = p->key_eq(src, chunk);
    PiXiuStr_free(src);
    if (!eq) return -5;
    int n = p->len;
    if (n > cap) return -2;
    memcpy(out, p->data, (size_t)n);
    *idx = (uint32_t)ci;
    return n;
}

// PiXiuCtrl::iter: drains every yielded generator into out (CSR offsets in off[]).
// Returns the record count, -1 for a NULL generator, -2 on overflow.
int refx_iter(const uint8_t *prefix, int plen, uint8_t *out, int cap, uint64_t *off, int max_recs) {
    CBTGen *g = g_ctrl.iter((uint8_t *)prefix, plen);
    if (g == nullptr) return -1;
    PXSGen *rv = nullptr;
    int n = 0;
    uint64_t d = 0;
    off[0] = 0;
    while (g->operator()(rv)) {
        if (n >= max_recs) return -2;
        int m = drain(rv, out + d, (int)(cap - d));
        if (m < 0) return -2;
        d += (uint64_t)m;
        off[++n] = d;
    }
    CBTGen_free(g);
    return n;
}

// PiXiuStr::parse(from,to) of record `idx` of the CURRENT chunk (PiXiuStr.cpp:166).
int refx_parse_current(int idx, int from, int to, uint8_t *out, int cap) {
    PiXiuChunk *c = g_ctrl.st.cbt_chunk;
    return drain(c->getitem(idx)->parse(from, to, c), out, cap);
}

// PiXiuStr_init / PiXiuStr_init_key (PiXiuStr.cpp:8-14).
int refx_escape(const uint8_t *src, int n, int is_key, uint8_t *out) {
    PiXiuStr *p = is_key ? PiXiuStr_init_key((uint8_t *)src, n) : PiXiuStr_init((uint8_t *)src, n);
    int len = p->len;
    memcpy(out, p->data, (size_t)len);
    PiXiuStr_free(p);
    return len;
}

// Raw stream encoder (PiXiuStr.cpp:16-118): feed n messages between ON and OFF.
int refx_stream(int n, const int *cmd, const int *pos, const uint8_t *val, uint8_t *out, int cap) {
    PXSMsg m;
    memset(&m, 0, sizeof m);
    m.chunk_idx_Cmd = PXS_STREAM_ON;
    PiXiuStr_init_stream(m);
    for (int i = 0; i < n; ++i) {
        m.chunk_idx_Cmd = cmd[i];
        m.pxs_idx = pos[i];
        m.val = val[i];
        PiXiuStr_init_stream(m);
    }
    memset(&m, 0, sizeof m);
    m.chunk_idx_Cmd = PXS_STREAM_OFF;
    PiXiuStr *p = PiXiuStr_init_stream(m);
    int len = p->len;
    if (len > cap) { PiXiuStr_free(p); return -1; }
    memcpy(out, p->data, (size_t)len);
    PiXiuStr_free(p);
    return len;
}

// Whole-corpus driver used for golden vectors: records i in [0,n) are
// key = keys[koff[i] .. +klen[i]], value = vals[voff[i] .. +vlen[i]].
// Outputs the compressed bytes, chunk number and slot of every record and,
// if do_get, the compat getitem() stream of every key after all inserts.
int refx_run(int n,
             const uint8_t *keys, const uint64_t *koff, const uint32_t *klen,
             const uint8_t *vals, const uint64_t *voff, const uint32_t *vlen,
             uint8_t *comp, uint64_t comp_cap, uint64_t *comp_off,
             uint32_t *chunk_no, uint32_t *idx,
             int do_get, uint8_t *dec, uint64_t dec_cap, uint64_t *dec_off) {
    refx_init();
    uint64_t c = 0;
    comp_off[0] = 0;
    for (int i = 0; i < n; ++i) {
        refx_setitem(keys + koff[i], (int)klen[i], vals + voff[i], (int)vlen[i], &chunk_no[i], &idx[i]);
        int m = refx_last_comp(comp + c, (int)(comp_cap - c < 0x7fffffff ? comp_cap - c : 0x7fffffff));
        if (m < 0) return -1;
        c += (uint64_t)m;
        comp_off[i + 1] = c;
    }
    if (do_get) {
        uint64_t d = 0;
        dec_off[0] = 0;
        for (int i = 0; i < n; ++i) {
            uint64_t room = dec_cap - d;
            int m = refx_getitem(keys + koff[i], (int)klen[i], dec + d, (int)(room < 0x7fffffff ? room : 0x7fffffff));
            if (m == -2) return -2;
            if (m < 0) m = 0;  // NULL getitem: recorded as empty
            d += (uint64_t)m;
            dec_off[i + 1] = d;
        }
    }
    return 0;
}

}  // extern "C"

// ---- debugging aid: dump the live GST as text (children in byte order)
#include <string>
static void dump_node(STNode *n, int depth, std::string &s) {
    for (int c = 0; c < 256; ++c) {
        STNode *k = n->get_sub((uint8_t)c);
        if (!k) continue;
        char buf[96];
        snprintf(buf, sizeof buf, "%*s[%d] d%u %u..%u%s\n", depth * 2, "", c, (unsigned)k->chunk_idx,
                 (unsigned)k->from, (unsigned)k->to, k->subs.root ? "" : " leaf");
        s += buf;
        dump_node(k, depth + 1, s);
    }
}
extern "C" int refx_dump_tree(char *out, int cap) {
    std::string s;
    dump_node(g_ctrl.st.root, 0, s);
    if ((int)s.size() + 1 > cap) return -1;
    memcpy(out, s.c_str(), s.size() + 1);
    return (int)s.size();
}

// Decode queries against a caller-supplied chunk of compressed records (for the
// decoder known-answer tests, e.g. PiXiuStr.cpp:356-413, which build chunks by hand).
extern "C" int refx_decode_chunk(int n, const uint8_t *comp, const uint64_t *off, int idx, int from, int to,
                                 uint8_t *out, int cap) {
    PiXiuChunk *c = PiXiuChunk_init();
    for (int i = 0; i < n; ++i) {
        int len = (int)(off[i + 1] - off[i]);
        PiXiuStr *p = (PiXiuStr *)malloc(sizeof(PiXiuStr) + (size_t)len + 8);
        p->len = (uint16_t)len;
        memcpy(p->data, comp + off[i], (size_t)len);
        c->strs[i] = p;
    }
    c->used_num = (uint16_t)n;
    int r = drain(c->getitem(idx)->parse(from, to, c), out, cap);
    PiXiuChunk_free(c);
    return r;
}
