// tools/proto/span_count.cpp — analysis prototype (not shipped, not a test).
//
// How many literal spans does a record's expansion resolve to?  Reads chunks dumped as
// [nrec][comp_len, doc_len, comp bytes]... (oracle-compressed) and maps every output
// byte of the exact and of the compat (PXSGen) expansion to the compressed byte it is
// copied from; a span is a maximal run of consecutive source addresses.  Same decode
// rules as oracle/pxo.cpp (compat_parse / exact_expand), restated over addresses.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <vector>
#include <algorithm>

typedef std::vector<uint8_t> Bytes;
typedef std::vector<uint32_t> Addr;
static const uint8_t kEsc = 251, kKeyEnd = 0, kValEnd = 2;

struct Chunk {
    std::vector<Bytes> recs;
    std::vector<uint32_t> base;  // global address of each record's first byte
    std::vector<Addr> exact;
    std::vector<int> st;
};

static int rd16(const Bytes &d, size_t i) { return d[i] | (d[i + 1] << 8); }
struct Ref { int idx, from, to; };
static Ref read_ref(const Bytes &d, size_t &i) {
    Ref r;
    uint8_t s = d[i + 1];
    if (s == 1) { r.idx = rd16(d, i + 2); r.to = rd16(d, i + 4); r.from = rd16(d, i + 6); i += 7; }
    else { r.idx = rd16(d, i + 2); r.to = rd16(d, i + 4); r.from = (uint16_t)(r.to - s); i += 5; }
    return r;
}

static const Addr &exact(Chunk &ch, int r) {
    if (ch.st[r] == 2) return ch.exact[r];
    ch.st[r] = 1;
    const Bytes &d = ch.recs[r];
    Addr out;
    for (size_t i = 0; i < d.size(); ++i) {
        if (d[i] != kEsc) { out.push_back(ch.base[r] + i); continue; }
        uint8_t nx = d[i + 1];
        if (nx == kKeyEnd || nx == kEsc || nx == kValEnd) {
            out.push_back(ch.base[r] + i); out.push_back(ch.base[r] + i + 1); ++i;
        } else if (nx == 1 || nx > 6) {
            Ref f = read_ref(d, i);
            if (f.idx == r) for (int k = f.from; k < f.to; ++k) out.push_back(out[k]);
            else { const Addr &s = exact(ch, f.idx); out.insert(out.end(), s.begin() + f.from, s.begin() + f.to); }
        }
    }
    ch.exact[r] = out;
    ch.st[r] = 2;
    return ch.exact[r];
}

struct Sink { Addr out; size_t limit = (size_t)-1; bool full(size_t cap) const { return out.size() >= std::min(cap, limit); } };

static void compat(const Chunk &ch, int self, int from, int to, Sink &s, size_t cap, int depth) {
    if (depth > 4096) throw std::runtime_error("depth");
    const Bytes &d = ch.recs[self];
    const int len = to - from;
    int src = 0, ret = 0;
    for (size_t i = 0; ret < len && i < d.size(); ++i) {
        uint8_t c = d[i];
        if (c != kEsc) {
            if (src >= from) { if (s.full(cap)) return; s.out.push_back(ch.base[self] + i); ++ret; }
            ++src;
            continue;
        }
        uint8_t nx = d[i + 1];
        if (nx == kKeyEnd || nx == kEsc || nx == kValEnd) {
            for (int h = 0; h < 2; ++h) {
                if (src >= from) { if (s.full(cap)) return; s.out.push_back(ch.base[self] + i + h); ++ret; }
                ++src;
            }
            ++i;
        } else if (nx == 1 || nx > 6) {
            Ref r = read_ref(d, i);
            int supply = r.to - r.from;
            if (src - 1 + supply >= from) {
                int sf = r.from + std::max(0, from - src);
                int stt = std::min(r.to, sf + (len - ret));
                if (sf < ret && ret < stt && r.idx == self) {
                    size_t start = s.out.size(), n = (size_t)(stt - sf);
                    while (s.out.size() - start != n) {
                        size_t before = s.out.size();
                        compat(ch, self, sf, ret, s, std::min(cap, start + n), depth + 1);
                        if (s.full(cap)) return;
                        if (s.out.size() == before) throw std::runtime_error("hang");
                    }
                } else {
                    compat(ch, r.idx, sf, stt, s, cap, depth + 1);
                    if (s.full(cap)) return;
                }
                ret += stt - sf;
            }
            src += supply;
        }
    }
}

// top-level segments (the runtime's SegEnt/LaneEnt entries): plain runs + record tokens
static size_t segments(const Bytes &d) {
    size_t n = 0;
    bool plain = false;
    for (size_t i = 0; i < d.size(); ++i) {
        if (d[i] == kEsc && i + 1 < d.size() && (d[i + 1] == 1 || d[i + 1] > 6)) {
            n += 1 + plain;
            plain = false;
            i += d[i + 1] == 1 ? 7 : 5;
            continue;
        }
        if (d[i] == kEsc) ++i;
        plain = true;
    }
    return n + plain + 1;
}

// 32-byte output tiles (the gather's unit): source loads as k_gather issues them (one
// unaligned 16-byte load per span piece inside the tile, a second for a piece over 16 bytes)
// against 16-byte windows covering the tile's source bytes greedily (one load serving every
// span whose bytes fall inside it)
static void tile_loads(const Addr &a, size_t &pieces, size_t &windows, size_t &tiles) {
    for (size_t t0 = 0; t0 < a.size(); t0 += 32) {
        const size_t t1 = std::min(a.size(), t0 + 32);
        ++tiles;
        size_t k = t0;
        std::vector<uint32_t> src;
        while (k < t1) {
            size_t e = k + 1;
            while (e < t1 && a[e] == a[e - 1] + 1) ++e;
            pieces += (e - k) > 16 ? 2 : 1;
            for (size_t q = k; q < e; ++q) src.push_back(a[q]);
            k = e;
        }
        std::sort(src.begin(), src.end());
        size_t i = 0;
        while (i < src.size()) {
            const uint32_t w = src[i];
            ++windows;
            while (i < src.size() && src[i] < w + 16) ++i;
        }
    }
}

static size_t spans(const Addr &a) {
    size_t n = 0;
    for (size_t k = 0; k < a.size(); ++k) n += (k == 0 || a[k] != a[k - 1] + 1);
    return n;
}

int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    size_t segs = 0, chunks = 0, recs = 0, comp = 0, out_e = 0, out_c = 0, sp_e = 0, sp_c = 0, differ = 0, maxsp = 0;
    size_t t_pieces = 0, t_windows = 0, t_tiles = 0;
    uint32_t nrec;
    while (fread(&nrec, 4, 1, f) == 1) {
        Chunk ch;
        uint32_t g = 0;
        for (uint32_t r = 0; r < nrec; ++r) {
            uint32_t cl, dl;
            if (fread(&cl, 4, 1, f) != 1 || fread(&dl, 4, 1, f) != 1) return 1;
            Bytes b(cl);
            if (fread(b.data(), 1, cl, f) != cl) return 1;
            ch.recs.push_back(b);
            ch.base.push_back(g);
            g += cl;
        }
        ch.exact.resize(nrec);
        ch.st.assign(nrec, 0);
        for (uint32_t r = 0; r < nrec; ++r) {
            const Addr &e = exact(ch, (int)r);
            Sink s;
            s.limit = 65535;
            compat(ch, (int)r, 0, 65535, s, (size_t)-1, 0);
            size_t a = spans(e), b = spans(s.out);
            tile_loads(s.out, t_pieces, t_windows, t_tiles);
            sp_e += a; sp_c += b; out_e += e.size(); out_c += s.out.size();
            differ += s.out != e;
            maxsp = std::max(maxsp, b);
            segs += segments(ch.recs[r]);
        }
        chunks++; recs += nrec; comp += g;
    }
    printf("%s: chunks %zu recs %zu comp %zu B | exact out %zu B spans %zu (%.1f B/span) | compat out %zu B spans %zu "
           "(%.1f B/span, max %zu/rec) | compat!=exact %zu | span table @8B = %.1f%% of comp | segments %zu (@48B = %.1f%%)\n",
           argv[1], chunks, recs, comp, out_e, sp_e, (double)out_e / sp_e, out_c, sp_c, (double)out_c / sp_c, maxsp,
           differ, 100.0 * 8 * sp_c / comp, segs, 100.0 * 48 * segs / comp);
    printf("compat tiles %zu: span-piece loads %zu (%.2f per tile), 16-byte window loads %zu (%.2f per tile, %.1f%% of the pieces)\n",
           t_tiles, t_pieces, (double)t_pieces / t_tiles, t_windows, (double)t_windows / t_tiles, 100.0 * t_windows / t_pieces);
}
