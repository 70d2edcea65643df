// oracle/pxo.cpp — TEST INFRASTRUCTURE ONLY (see pxo.h).  Never linked into the
// product; tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it
// as the checker / CPU baseline ("kind": "port").
//
// A clean-room restatement of the reference's hot path, written from its observable
// behaviour — each piece cites what it follows:
//   escape / doc assembly ........ PiXiuStr.cpp:228-271, PiXiuCtrl.cpp:31-44
//   stream encoder ............... PiXiuStr.cpp:16-118 (2-message 251 look-ahead,
//                                  run > 6 -> 6 B small / 8 B big record, len byte 251 alias kept)
//   Ukkonen GST step ............. SuffixTree.cpp:144-289 (active point, split/grow,
//                                  suffix links, canonisation), reset at SuffixTree.cpp:85-89
//   pool accounting + rotation ... MemPool.cpp:7-37 (65,535 x 8 B pools; node = 5 blocks,
//                                  child-map entry = 3 blocks), PiXiuCtrl.cpp:13-25
//   compat decoder ............... PiXiuStr.h:129-198 (rescan-from-token-0 recursion,
//                                  relative-cursor overlap test, per-token length check)
//   exact decoder ................ the same token grammar with LZ semantics on the
//                                  absolute cursor (what the encoder meant)
// The child map is an ordered map (a sorted vector here) exactly like the reference's
// ScapegoatTree in semantics, so this is the same algorithm the reference runs, minus
// its process-global state: every pxo_shard is independent.
#include "pxo.h"

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace {

constexpr uint8_t kEsc = 251;
constexpr uint8_t kKeyEnd = 0;
constexpr uint8_t kValEnd = 2;
constexpr int kMaxDoc = 65535;
constexpr int kChunkSlots = 65535;
constexpr int kPoolBlocks = 65535;
constexpr int kNodeBlocks = 5;   // 40-byte tree node
constexpr int kEdgeBlocks = 3;   // 24-byte child-map entry
constexpr int kRotatePools = 2048;
constexpr uint32_t kNone = 0xffffffffu;
constexpr uint32_t kRoot = 0;
constexpr int kCmdOn = -1, kCmdOff = -2, kCmdPass = -3;
constexpr int kMaxDepth = 1 << 16;

struct Fail {
    int code;
};
int g_fail_line = 0;
std::vector<int> g_trace;  // debugging aid: per-byte message log
bool g_trace_on = false;
inline void trace(int cmd, int pos, uint8_t v) {
    if (g_trace_on) { g_trace.push_back(cmd); g_trace.push_back(pos); g_trace.push_back(v); }
}
#define FAIL(c) (g_fail_line = __LINE__, Fail{c})

using Bytes = std::vector<uint8_t>;

void escape_append(const uint8_t *src, int n, bool key, Bytes &out) {
    for (int i = 0; i < n; ++i) {
        out.push_back(src[i]);
        if (src[i] == kEsc) out.push_back(kEsc);
    }
    if (key) {
        out.push_back(kEsc);
        out.push_back(kKeyEnd);
    }
}

// Doc assembly: esc(k)+[251,0] (+ esc(v)+[251,2]).  Empty keys and docs longer
// than 65,535 B are asserts in the reference (UB in Release) -> error here.
int assemble_doc(const uint8_t *k, int klen, const uint8_t *v, int vlen, Bytes &doc) {
    doc.clear();
    if (klen <= 0) return PXO_EINVAL;
    escape_append(k, klen, true, doc);
    if (vlen > 0) {
        escape_append(v, vlen, true, doc);
        doc.back() = kValEnd;
    }
    if ((int)doc.size() > kMaxDoc) return PXO_EINVAL;
    return 0;
}

// ---------------------------------------------------------------- stream encoder
struct Msg {
    int cmd;
    int pos;
    uint8_t val;
};

class StreamEncoder {
  public:
    // returns 1 when an OFF produced a result in `result`
    int feed(Msg m, Bytes *result) {
        for (;;) {
            if ((held_ == 0 && m.val == kEsc) || held_ == 1) {
                hold_[held_++] = m;
                return 0;
            }
            if (held_ == 2) {
                bool both_c = hold_[0].cmd >= 0 && hold_[1].cmd >= 0;
                bool both_p = hold_[0].cmd == kCmdPass && hold_[1].cmd == kCmdPass;
                for (int k = 0; k < 2; ++k) {
                    Msg h = hold_[k];
                    if (!(both_c || both_p)) h.cmd = kCmdPass;
                    act(h, nullptr);
                }
                held_ = 0;
                continue;
            }
            return act(m, result);
        }
    }

  private:
    int act(const Msg &m, Bytes *result) {
        switch (m.cmd) {
        case kCmdOn:
            out_.clear();
            run_ = 0;
            return 0;
        case kCmdPass:
            flush_run();
            out_.push_back(m.val);
            return 0;
        case kCmdOff:
            flush_run();
            if (result) *result = out_;
            return 1;
        default:
            run_idx_ = m.cmd;
            run_to_ = m.pos + 1;
            ++run_;
            out_.push_back(m.val);
            return 0;
        }
    }

    void put16(int v) {
        out_.push_back((uint8_t)(v & 0xff));
        out_.push_back((uint8_t)((v >> 8) & 0xff));
    }

    void flush_run() {
        if (run_ <= 0) return;
        if (run_ > 6) {
            out_.resize(out_.size() - (size_t)run_);
            out_.push_back(kEsc);
            if (run_ > 255) {
                out_.push_back(1);
                put16(run_idx_);
                put16(run_to_);
                put16(run_to_ - run_);
            } else {
                out_.push_back((uint8_t)run_);
                put16(run_idx_);
                put16(run_to_);
            }
        }
        run_ = 0;
    }

    Bytes out_;
    int run_ = 0, run_idx_ = 0, run_to_ = 0;
    Msg hold_[2] = {};
    int held_ = 0;
};

// ---------------------------------------------------------------- Ukkonen GST
struct GNode {
    uint32_t link;
    uint16_t doc, from, to;
    std::vector<std::pair<uint8_t, uint32_t>> kids;  // ordered child map
};

class Gst {
  public:
    Gst() { clear(); }

    void clear() {
        nodes_.clear();
        docs_.clear();
        pools_ = 0;
        used_ = 0;
        pool_open_ = false;
        charge(kNodeBlocks);
        nodes_.push_back(GNode{kRoot, 0, 0, 0, {}});
        reset_active();
    }

    int pools() const { return pools_; }
    int used_blocks() const { return used_; }
    long ub_reads() const { return ub_reads_; }
    size_t num_docs() const { return docs_.size(); }

    // SuffixTree::setitem (SuffixTree.cpp:291-304): returns the compressed doc.
    Bytes add_doc(const Bytes &doc) {
        cur_ = (uint16_t)docs_.size();
        docs_.push_back(doc);
        Bytes res;
        enc_.feed(Msg{kCmdOn, 0, 0}, nullptr);
        const Bytes &d = docs_.back();
        for (size_t i = 0; i < d.size(); ++i) step(d[i]);
        if (!enc_.feed(Msg{kCmdOff, 0, 0}, &res)) throw FAIL(PXO_ECORRUPT);
        reset_active();
        return res;
    }

    // debugging aid: the tree as text, children in byte order
    void dump(uint32_t n, int depth, std::string &s) const {
        for (const auto &kv : nodes_[n].kids) {
            const GNode &k = nodes_[kv.second];
            char buf[96];
            snprintf(buf, sizeof buf, "%*s[%d] d%u %u..%u%s\n", depth * 2, "", (int)kv.first, (unsigned)k.doc,
                     (unsigned)k.from, (unsigned)k.to, k.kids.empty() ? " leaf" : "");
            s += buf;
            dump(kv.second, depth + 1, s);
        }
    }

  private:
    void reset_active() {
        remainder_ = 0;
        counter_ = 0;
        act_node_ = kRoot;
        act_doc_ = act_direct_ = act_off_ = 0;
    }

    void charge(int blocks) {  // MemPool::p_malloc block accounting
        if (!pool_open_) {
            pool_open_ = true;
            ++pools_;
            used_ = 0;
        }
        if (blocks > kPoolBlocks - used_) {
            ++pools_;
            used_ = 0;
        }
        used_ += blocks;
    }

    uint8_t text(uint32_t doc, uint32_t pos) const {
        if (doc >= docs_.size() || pos >= docs_[doc].size()) throw FAIL(PXO_ECORRUPT);
        return docs_[doc][pos];
    }

    // A read the reference makes through a stale (act_chunk_idx, act_direct) pair.
    // It can run past the end of that doc (heap bytes: undefined behaviour in the
    // reference).  Such a read is modelled as a value matching no byte (-1) and
    // counted in ub_reads so tests can tell "reference UB" apart from a mismatch.
    int stale_text(uint32_t doc, uint32_t pos) {
        if (doc >= docs_.size()) throw FAIL(PXO_ECORRUPT);
        if (pos >= docs_[doc].size()) {
            ++ub_reads_;
            return -1;
        }
        return docs_[doc][pos];
    }

    uint8_t head(uint32_t n) const { return text(nodes_[n].doc, nodes_[n].from); }

    uint32_t child(uint32_t n, uint8_t c) const {
        const auto &k = nodes_[n].kids;
        auto it = std::lower_bound(k.begin(), k.end(), std::make_pair(c, (uint32_t)0),
                                   [](const std::pair<uint8_t, uint32_t> &a,
                                      const std::pair<uint8_t, uint32_t> &b) { return a.first < b.first; });
        if (it != k.end() && it->first == c) return it->second;
        return kNone;
    }

    uint32_t must_child(uint32_t n, uint8_t c) const {
        uint32_t r = child(n, c);
        if (r == kNone) throw FAIL(PXO_ECORRUPT);  // the reference would dereference NULL
        return r;
    }

    // set_sub: insert (charges one map entry) or replace an equal key (free)
    void set_child(uint32_t n, uint32_t kid) {
        uint8_t c = head(kid);
        auto &k = nodes_[n].kids;
        auto it = std::lower_bound(k.begin(), k.end(), std::make_pair(c, (uint32_t)0),
                                   [](const std::pair<uint8_t, uint32_t> &a,
                                      const std::pair<uint8_t, uint32_t> &b) { return a.first < b.first; });
        if (it != k.end() && it->first == c) {
            it->second = kid;
            return;
        }
        charge(kEdgeBlocks);
        k.insert(it, std::make_pair(c, kid));
    }

    uint32_t new_node(uint16_t doc, uint16_t from, uint16_t to) {
        charge(kNodeBlocks);
        nodes_.push_back(GNode{kRoot, doc, from, to, {}});
        return (uint32_t)nodes_.size() - 1;
    }

    bool is_inner(uint32_t n) const { return n != kRoot && !nodes_[n].kids.empty(); }

    void emit_pass(uint8_t c) { trace(kCmdPass, 0, c); enc_.feed(Msg{kCmdPass, 0, c}, nullptr); }
    void emit_copy(int doc, int pos, uint8_t c) { trace(doc, pos, c); enc_.feed(Msg{doc, pos, c}, nullptr); }

    void at_root(uint8_t c, bool send) {
        uint32_t e = child(kRoot, c);
        if (e == kNone) {
            uint32_t leaf = new_node(cur_, counter_, (uint16_t)docs_[cur_].size());
            set_child(kRoot, leaf);
            --remainder_;
            if (send) emit_pass(c);
        } else {
            act_doc_ = nodes_[e].doc;
            act_direct_ = nodes_[e].from;
            ++act_off_;
            if (send) emit_copy(nodes_[e].doc, nodes_[e].from, c);
        }
    }

    // overflow_fix: walk the active point down whole edges of the current text
    uint32_t canonise() {
        const Bytes &t = docs_[cur_];
        int end = counter_;
        int begin = end - act_off_;
        uint32_t e = must_child(act_node_, t[counter_ - act_off_]);
        int supply;
        while (end - begin > (supply = nodes_[e].to - nodes_[e].from)) {
            act_node_ = e;
            begin += supply;
            act_off_ = (uint16_t)(act_off_ - supply);
            e = must_child(act_node_, t[begin]);
            act_direct_ = nodes_[e].from;
        }
        return e;
    }

    void grow(uint32_t e, uint32_t &last_inner) {
        uint32_t leaf = new_node(cur_, counter_, (uint16_t)docs_[cur_].size());
        --remainder_;
        GNode *en = &nodes_[e];
        bool e_leaf = (e != kRoot) && en->kids.empty();
        if ((e_leaf || en->to - en->from > 1) && en->from + act_off_ != en->to) {
            uint32_t in = new_node(en->doc, en->from, (uint16_t)(en->from + act_off_));
            en = &nodes_[e];
            if (last_inner != kNone) nodes_[last_inner].link = in;
            last_inner = in;
            set_child(act_node_, in);  // replaces e under the same first byte
            en->from = nodes_[in].to;
            set_child(in, e);
            set_child(in, leaf);
        } else {
            if (last_inner != kNone) nodes_[last_inner].link = e;
            last_inner = e;
            set_child(e, leaf);
        }
    }

    // s_insert_char (SuffixTree.cpp:144-289)
    void step(uint8_t c) {
        if (g_trace_on) {  // debugging aid: state at each doc position
            trace(-100 - (int)counter_, (int)act_node_, act_doc_);
            trace(act_direct_, act_off_, (uint8_t)0);
            g_trace.back() = remainder_;
            trace((int)nodes_.size(), pools_, (uint8_t)0);
            g_trace.back() = used_;
        }
        ++remainder_;
        if (act_node_ == kRoot && act_off_ == 0) {
            at_root(c, true);
        } else {
            int key = stale_text(act_doc_, act_direct_);
            if (key < 0) throw FAIL(PXO_ECORRUPT);  // reference: get_sub(garbage) -> NULL
            uint32_t e = must_child(act_node_, (uint8_t)key);
            uint32_t nx;
            if (nodes_[e].from + act_off_ == nodes_[e].to && (nx = child(e, c)) != kNone) {
                act_node_ = e;
                act_doc_ = nodes_[nx].doc;
                act_direct_ = nodes_[nx].from;
                act_off_ = 1;
                emit_copy(nodes_[nx].doc, nodes_[nx].from, c);
            } else if (nodes_[e].from + act_off_ < nodes_[e].to &&
                       (int)c == stale_text(act_doc_, nodes_[e].from + act_off_)) {
                // NB: the reference reads the *active* doc here (edge_pxs is
                // strs[act_chunk_idx], SuffixTree.cpp:171,184), not the edge's own doc;
                // the two differ once canonisation has moved act_direct without
                // act_chunk_idx (SuffixTree.cpp:232-246).  Kept bit-for-bit.
                emit_copy(nodes_[e].doc, nodes_[e].from + act_off_, c);
                ++act_off_;
            } else {
                emit_pass(c);
                uint32_t last_inner = kNone;
                while (remainder_ > 0) {
                    grow(e, last_inner);
                    if (!is_inner(act_node_)) {
                        --act_off_;
                        ++act_direct_;
                        if (act_off_ > 0) {
                            e = canonise();
                        } else {
                            at_root(c, false);
                            break;
                        }
                    } else {
                        act_node_ = nodes_[act_node_].link;
                        e = canonise();
                    }
                    if (nodes_[e].from + act_off_ == nodes_[e].to && (nx = child(e, c)) != kNone) {
                        act_node_ = e;
                        act_doc_ = nodes_[nx].doc;
                        act_direct_ = nodes_[nx].from;
                        act_off_ = 1;
                        if (last_inner != kNone) nodes_[last_inner].link = act_node_;
                        break;
                    } else if (nodes_[e].from + act_off_ < nodes_[e].to &&
                               c == text(nodes_[e].doc, nodes_[e].from + act_off_)) {
                        ++act_off_;
                        break;
                    }
                }
            }
        }
        ++counter_;
    }

    std::vector<GNode> nodes_;
    std::vector<Bytes> docs_;
    StreamEncoder enc_;
    int pools_ = 0, used_ = 0;
    bool pool_open_ = false;
    uint32_t act_node_ = kRoot;
    uint16_t act_doc_ = 0, act_direct_ = 0, act_off_ = 0;
    uint16_t counter_ = 0, cur_ = 0;
    int remainder_ = 0;
    long ub_reads_ = 0;
};

// ---------------------------------------------------------------- decoders
struct Chunk {
    std::vector<Bytes> recs;
    std::vector<uint8_t> dead;
    int used = 0;   // PiXiuChunk::used_num: records placed minus deleted (PiXiuStr.h:76)
    int total = 0;  // PiXiuChunk::total_num: set when the chunk is closed (PiXiuCtrl.cpp:15)
    std::vector<Bytes> exact;          // memo of exact expansions
    std::vector<uint8_t> exact_state;  // 0 none, 1 in progress, 2 done
};

inline int rd16(const Bytes &d, size_t i) {
    if (i + 1 >= d.size()) throw FAIL(PXO_ECORRUPT);
    return d[i] | (d[i + 1] << 8);
}

struct RecordRef {
    int idx, from, to;
};

// Decode the record token at d[i] (d[i] == 251, d[i+1] == 1 or > 6); advances i
// to the token's last byte, exactly like the reference's `i += sizeof(...) - 1`.
RecordRef read_record(const Bytes &d, size_t &i) {
    RecordRef r;
    uint8_t sign = d[i + 1];
    if (sign == 1) {
        r.idx = rd16(d, i + 2);
        r.to = rd16(d, i + 4);
        r.from = rd16(d, i + 6);
        i += 7;
    } else {
        r.idx = rd16(d, i + 2);
        r.to = rd16(d, i + 4);
        r.from = (uint16_t)(r.to - sign);
        i += 5;
    }
    return r;
}

// Where decoded bytes go.  `limit` is the consumer's hard stop (it stops pulling);
// with key_stop set the consumer stops right after the key terminator 251,0 as
// PXSG_SEE_KEY_BREAK (PiXiuStr.h:23-30) does.
struct Sink {
    Bytes out;
    size_t limit = (size_t)-1;
    bool key_stop = false;
    bool spec = false;
    bool key_end_seen = false;

    bool full(size_t cap) const { return out.size() >= std::min(cap, limit); }
    void put(uint8_t b) {
        out.push_back(b);
        if (!key_stop) return;
        if (!spec && b == kEsc) {
            spec = true;
        } else if (spec) {
            if (b == kKeyEnd) {
                key_end_seen = true;
                limit = out.size();
            } else {
                spec = false;
            }
        }
    }
};

// PXSGen semantics (PiXiuStr.h:129-198) in push form.  `cap` is the absolute
// output size at which the innermost enclosing periodic loop stops pulling.
void compat_parse(const Chunk &ch, uint32_t self, int from, int to, Sink &s, size_t cap, int depth) {
    if (self >= ch.recs.size()) throw FAIL(PXO_ECORRUPT);
    if (depth > kMaxDepth) throw FAIL(PXO_EHANG);
    const Bytes &d = ch.recs[self];
    const int len = to - from;
    int src = 0, ret = 0;
    for (size_t i = 0; ret < len && i < d.size(); ++i) {
        uint8_t c = d[i];
        if (c != kEsc) {
            if (src >= from) {
                if (s.full(cap)) return;
                s.put(c);
                ++ret;
            }
            ++src;
            continue;
        }
        if (i + 1 >= d.size()) throw FAIL(PXO_ECORRUPT);
        uint8_t nx = d[i + 1];
        if (nx == kKeyEnd || nx == kEsc || nx == kValEnd) {
            // both halves are written with only the src test: the per-token
            // `ret < len` check lets a range ending mid-pair over-yield one byte
            for (int half = 0; half < 2; ++half) {
                if (src >= from) {
                    if (s.full(cap)) return;
                    s.put(half ? nx : kEsc);
                    ++ret;
                }
                ++src;
            }
            ++i;
        } else if (nx == 1 || nx > 6) {
            RecordRef r = read_record(d, i);
            int supply = r.to - r.from;
            if (src - 1 + supply >= from) {
                int sub_from = r.from + std::max(0, from - src);
                int sub_to = std::min(r.to, sub_from + (len - ret));
                // overlap test on the RELATIVE cursor `ret` (reference bug, kept)
                if (sub_from < ret && ret < sub_to && (uint32_t)r.idx == self) {
                    const size_t start = s.out.size();
                    const size_t n = (size_t)(sub_to - sub_from);
                    while (s.out.size() - start != n) {
                        size_t before = s.out.size();
                        compat_parse(ch, self, sub_from, ret, s, std::min(cap, start + n), depth + 1);
                        if (s.full(cap)) return;
                        if (s.out.size() == before) throw FAIL(PXO_EHANG);
                    }
                } else {
                    compat_parse(ch, (uint32_t)r.idx, sub_from, sub_to, s, cap, depth + 1);
                    if (s.full(cap)) return;
                }
                ret += sub_to - sub_from;
            }
            src += supply;
        }
        // 251 followed by 3..6 is an assert(false) in the reference; with NDEBUG the
        // 251 is consumed and nothing is written (the next byte is re-read as a token).
    }
}

const Bytes &exact_expand(Chunk &ch, uint32_t r, int depth) {
    if (r >= ch.recs.size()) throw FAIL(PXO_ECORRUPT);
    if (ch.exact.size() < ch.recs.size()) {
        ch.exact.resize(ch.recs.size());
        ch.exact_state.resize(ch.recs.size(), 0);
    }
    if (ch.exact_state[r] == 2) return ch.exact[r];
    if (ch.exact_state[r] == 1 || depth > kMaxDepth) throw FAIL(PXO_ECORRUPT);
    ch.exact_state[r] = 1;
    const Bytes &d = ch.recs[r];
    Bytes out;
    for (size_t i = 0; i < d.size(); ++i) {
        uint8_t c = d[i];
        if (c != kEsc) {
            out.push_back(c);
            continue;
        }
        if (i + 1 >= d.size()) throw FAIL(PXO_ECORRUPT);
        uint8_t nx = d[i + 1];
        if (nx == kKeyEnd || nx == kEsc || nx == kValEnd) {
            out.push_back(kEsc);
            out.push_back(nx);
            ++i;
        } else if (nx == 1 || nx > 6) {
            RecordRef rr = read_record(d, i);
            if (rr.to < rr.from) throw FAIL(PXO_ECORRUPT);
            if ((uint32_t)rr.idx == r) {  // LZ self-copy, may overlap its own output
                for (int k = rr.from; k < rr.to; ++k) {
                    if ((size_t)k >= out.size()) throw FAIL(PXO_ECORRUPT);
                    out.push_back(out[(size_t)k]);
                }
            } else {
                const Bytes &src = exact_expand(ch, (uint32_t)rr.idx, depth + 1);
                if ((size_t)rr.to > src.size()) throw FAIL(PXO_ECORRUPT);
                out.insert(out.end(), src.begin() + rr.from, src.begin() + rr.to);
            }
        }
    }
    ch.exact[r] = std::move(out);
    ch.exact_state[r] = 2;
    return ch.exact[r];
}

// ---------------------------------------------------------------- crit-bit index
// Restates CritBitTree.cpp:13-269: a crit-bit trie over escaped docs whose
// comparisons run against the COMPAT-decoded stored record (so decoder quirks
// shape the trie exactly as in the reference).
struct Leaf {
    uint32_t chunk, idx;
};
struct CbtRef {
    int32_t inner = -1;  // >= 0: inner node index, else a leaf
    Leaf leaf{0, 0};
};
struct CbtInner {
    CbtRef kid[2];
    uint16_t diff_at;
    uint8_t mask;
};

inline int crit_dir(uint8_t mask, uint8_t byte) { return (1 + (mask | byte)) >> 8; }

}  // namespace

// ---------------------------------------------------------------- shard
struct pxo_shard {
    Gst gst;
    std::vector<Chunk> chunks;
    std::vector<CbtInner> cbt;
    std::vector<int32_t> cbt_free;
    bool has_root = false;
    CbtRef root;

    // Glob_Reinsert_Chunk (PiXiuStr.cpp:4), per instance here: the last chunk a delete
    // left under 80 % of PXC_STR_NUM live records (PiXiuStr.cpp:178-187), or -1
    int glob = -1;

    pxo_shard() { chunks.emplace_back(); }

    bool rotation_due() const { return gst.pools() >= kRotatePools || gst.num_docs() == (size_t)kChunkSlots; }
    // SuffixTree::setitem into the live chunk
    void place(const Bytes &doc, uint32_t *chunk_no, uint32_t *idx) {
        Chunk &ch = chunks.back();
        ch.recs.push_back(gst.add_doc(doc));
        ch.dead.push_back(0);
        ch.used++;
        *chunk_no = (uint32_t)chunks.size() - 1;
        *idx = (uint32_t)ch.recs.size() - 1;
    }
    // PiXiuCtrl::setitem minus CritBit and reinsert: rotation check (PiXiuCtrl.cpp:13),
    // then SuffixTree::setitem (the encoder-only driver)
    void store(const Bytes &doc, uint32_t *chunk_no, uint32_t *idx) {
        if (rotation_due()) {
            gst.clear();
            chunks.emplace_back();
        }
        place(doc, chunk_no, idx);
    }

    // need_reinsert (PiXiuCtrl.cpp:7-8): live records under half of the closed total
    bool need_reinsert(int c) const { return chunks[(size_t)c].used < 0.5 * chunks[(size_t)c].total; }
    int live_chunk() const { return (int)chunks.size() - 1; }

    // PiXiuChunk::delitem (PiXiuStr.cpp:178-187)
    void chunk_delitem(const Leaf &l) {
        Chunk &ch = chunks[l.chunk];
        if (ch.dead[l.idx]) throw FAIL(PXO_ECORRUPT);  // the reference asserts
        ch.dead[l.idx] = 1;
        ch.used--;
        if (ch.used < 0.8 * kChunkSlots) glob = (int)l.chunk;
    }

    // PiXiuCtrl::setitem (PiXiuCtrl.cpp:12-47) with its reinsert triggers
    int ctrl_set(const Bytes &doc, bool reinsert, uint32_t *c, uint32_t *i) {
        if (rotation_due()) {
            const int last = live_chunk();
            chunks[(size_t)last].total = (int)gst.num_docs();
            gst.clear();
            chunks.emplace_back();
            if (need_reinsert(last)) {
                if (last == glob) glob = -1;
                reinsert_chunk(last, false);
            }
        }
        if (!reinsert && glob >= 0 && glob != live_chunk() && need_reinsert(glob)) reinsert_chunk(glob, true);
        place(doc, c, i);
        return index_insert(doc, Leaf{*c, *i});
    }

    // PiXiuCtrl::delitem's trigger (PiXiuCtrl.cpp:63-69), before the CritBit delete
    void delete_trigger() {
        if (glob >= 0 && glob != live_chunk() && need_reinsert(glob)) reinsert_chunk(glob, true);
    }

    // PiXiuCtrl::reinsert (PiXiuCtrl.cpp:88-114): every live record of chunk c, decoded
    // through PXSGen (compat), goes back in through setitem as a ready doc; the CritBit
    // replace deletes the old copy.  The loop visits all PXC_STR_NUM slots and the
    // reference asserts each is set (PiXiuStr.cpp:189-193): only a slot-full chunk is
    // well defined, and only that case is carried out (any other is a no-op here).
    // `via_glob`: called as reinsert(Glob_Reinsert_Chunk), whose reference argument the
    // final `chunk = NULL` clears.
    void reinsert_chunk(int c, bool via_glob) {
        if (chunks[(size_t)c].recs.size() != (size_t)kChunkSlots) return;
        const int curr = glob;
        for (uint32_t i = 0; i < (uint32_t)kChunkSlots; ++i) {
            if (chunks[(size_t)c].dead[i]) continue;
            Sink sk;
            sk.limit = (size_t)kMaxDoc;
            decode_into((uint32_t)c, i, 0, kMaxDoc, PXO_COMPAT, sk);
            uint32_t cc, ii;
            ctrl_set(sk.out, true, &cc, &ii);
        }
        Chunk &ch = chunks[(size_t)c];  // PiXiuChunk_free: the chunk's records are gone
        std::fill(ch.dead.begin(), ch.dead.end(), 1);
        ch.used = 0;
        glob = via_glob ? -1 : curr;
    }

    void decode_into(uint32_t c, uint32_t i, int from, int to, int mode, Sink &s) {
        if (mode == PXO_COMPAT) {
            compat_parse(chunks[c], i, from, to, s, (size_t)-1, 0);
        } else {
            const Bytes &e = exact_expand(chunks[c], i, 0);
            size_t a = std::min((size_t)from, e.size()), b = std::min((size_t)to, e.size());
            for (size_t k = a; k < b && !s.full((size_t)-1); ++k) s.put(e[k]);
        }
    }

    // compat-decoded prefix of a stored record up to (and incl.) its key terminator
    Bytes key_prefix(const Leaf &l) {
        Sink s;
        s.key_stop = true;
        decode_into(l.chunk, l.idx, 0, kMaxDoc, PXO_COMPAT, s);
        return std::move(s.out);
    }

    struct Best {
        int32_t grand = -1, pa = -1;
        int dir = 3;
        Leaf crit{0, 0};
    };

    Best best_match(const Bytes &q) const {  // find_best_match (CritBitTree.cpp:253-269)
        Best b;
        CbtRef p = root;
        while (p.inner >= 0) {
            const CbtInner &n = cbt[(size_t)p.inner];
            uint8_t byte = q.size() > n.diff_at ? q[n.diff_at] : 0;
            b.dir = crit_dir(n.mask, byte);
            b.grand = b.pa;
            b.pa = p.inner;
            p = n.kid[b.dir];
        }
        b.crit = p.leaf;
        return b;
    }


    int32_t new_inner() {
        if (!cbt_free.empty()) {
            int32_t r = cbt_free.back();
            cbt_free.pop_back();
            return r;
        }
        cbt.emplace_back();
        return (int32_t)cbt.size() - 1;
    }

    // CritBitTree::setitem (CritBitTree.cpp:13-105)
    int index_insert(const Bytes &doc, Leaf nl) {
        CbtRef nref;
        nref.leaf = nl;
        if (!has_root) {
            has_root = true;
            root = nref;
            return 0;
        }
        Best b = best_match(doc);
        Bytes crit = key_prefix(b.crit);
        // compare the crit stream with the raw doc until a difference or 251,0
        size_t k = 0;
        uint16_t diff_at = 0;
        uint8_t crit_rv = 0, src_rv = 0;
        bool spec = false;
        for (;;) {
            if (k >= crit.size()) break;  // crit stream exhausted: values stay stale
            crit_rv = crit[k];
            if (k >= doc.size()) break;
            src_rv = doc[k];
            ++k;
            if (crit_rv != src_rv) break;
            if (!spec && crit_rv == kEsc) {
                spec = true;
            } else if (spec) {
                if (crit_rv == kKeyEnd) {  // same key: replace (CBT_SET_REPLACE)
                    chunk_delitem(b.crit);
                    if (b.pa < 0) root = nref;
                    else cbt[(size_t)b.pa].kid[b.dir] = nref;
                    return 1;
                }
                spec = false;
            }
            ++diff_at;
        }
        if (spec) return 0;  // unreachable for well-formed streams (reference: no insert)
        uint8_t mask = crit_rv ^ src_rv;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask = (uint8_t)((mask & ~(mask >> 1)) ^ 0xff);
        uint8_t at = diff_at < doc.size() ? doc[diff_at] : 0;  // past the end: UB in the reference
        int dir = crit_dir(mask, at);
        int32_t in = new_inner();
        cbt[(size_t)in].diff_at = diff_at;
        cbt[(size_t)in].mask = mask;
        cbt[(size_t)in].kid[dir] = nref;
        // walk down to the insertion point
        int32_t parent = -1;
        int pdir = 0;
        CbtRef p = root;
        while (p.inner >= 0) {
            const CbtInner &n = cbt[(size_t)p.inner];
            if (n.diff_at > diff_at || (n.diff_at == diff_at && n.mask > mask)) break;
            uint8_t byte = doc.size() > n.diff_at ? doc[n.diff_at] : 0;
            pdir = crit_dir(n.mask, byte);
            parent = p.inner;
            p = n.kid[pdir];
        }
        CbtRef iref;
        iref.inner = in;
        if (parent < 0) root = iref;
        else cbt[(size_t)parent].kid[pdir] = iref;
        cbt[(size_t)in].kid[1 - dir] = p;
        return 0;
    }

    // CritBitTree::contains / delitem (CritBitTree.cpp:107-178): the crit record's decoded
    // stream is compared with the escaped key bytes until the key terminator.
    bool key_matches(const Bytes &q, const Leaf &l) {
        Bytes crit = key_prefix(l);
        bool spec = false;
        for (size_t k = 0; k < crit.size() && k < q.size() && crit[k] == q[k]; ++k) {
            uint8_t v = crit[k];
            if (!spec && v == kEsc) {
                spec = true;
            } else if (spec) {
                if (v == kKeyEnd) return true;
                spec = false;
            }
        }
        return false;
    }

    bool contains(const Bytes &q) {
        if (!has_root) return false;
        return key_matches(q, best_match(q).crit);
    }

    int remove(const Bytes &q) {  // 0 deleted, 1 CBT_DEL_NOT_FOUND
        if (!has_root) return 1;
        Best b = best_match(q);
        if (!key_matches(q, b.crit)) return 1;
        if (b.pa < 0) {
            has_root = false;
            root = CbtRef{};
        } else {
            CbtRef other = cbt[(size_t)b.pa].kid[1 - b.dir];
            if (b.grand < 0) {
                root = other;
            } else {
                CbtInner &g = cbt[(size_t)b.grand];
                g.kid[g.kid[0].inner == b.pa ? 0 : 1] = other;
            }
            cbt_free.push_back(b.pa);
        }
        chunk_delitem(b.crit);
        return 0;
    }

    // PiXiuStr::startswith (PiXiuStr.cpp:145-164): the record's compat stream begins
    // with `prefix` (escaped, no terminator)
    bool startswith(const Leaf &l, const Bytes &prefix) {
        Sink s;
        s.limit = prefix.size();
        decode_into(l.chunk, l.idx, 0, kMaxDoc, PXO_COMPAT, s);
        return s.out.size() == prefix.size() && std::equal(prefix.begin(), prefix.end(), s.out.begin());
    }

    // CritBitTree::iter / CBTGHelper / CBTGen (CritBitTree.h:55-157, CritBitTree.cpp:271-282):
    // follow the prefix's crit bits; once a node's diff_at reaches past the prefix the
    // whole subtree is taken (kid 0 before kid 1).  The first leaf reached is checked
    // with startswith; if it fails the generator yields NULL and CBTGen stops, else it
    // and every later leaf are yielded unchecked.  Returns false for an empty tree.
    bool iter(const Bytes &prefix, std::vector<Leaf> &out) {
        if (!has_root) return false;
        bool harvest = false;
        std::vector<std::pair<CbtRef, bool>> stack{{root, false}};
        while (!stack.empty()) {
            auto [ref, include_all] = stack.back();
            stack.pop_back();
            if (ref.inner < 0) {
                if (!harvest && !startswith(ref.leaf, prefix)) break;
                harvest = true;
                out.push_back(ref.leaf);
                continue;
            }
            const CbtInner &n = cbt[(size_t)ref.inner];
            uint8_t crit = prefix.size() > n.diff_at ? prefix[n.diff_at] : 0;
            int direct = crit_dir(n.mask, crit);
            if (!include_all && n.diff_at >= prefix.size()) include_all = true;
            if (include_all) {
                stack.push_back({n.kid[1], true});
                stack.push_back({n.kid[0], true});
            } else {
                stack.push_back({n.kid[direct], false});
            }
        }
        return true;
    }

    // CritBitTree::getitem + key_eq (CritBitTree.cpp:180-196; PiXiuStr.cpp:129-143)
    bool lookup(const Bytes &q, Leaf *out) {
        if (!has_root) return false;
        Best b = best_match(q);
        Bytes crit = key_prefix(b.crit);
        bool spec = false;
        for (size_t k = 0; k < crit.size() && k < q.size() && crit[k] == q[k]; ++k) {
            uint8_t v = crit[k];
            if (!spec && v == kEsc) {
                spec = true;
            } else if (spec) {
                if (v == kKeyEnd) {
                    *out = b.crit;
                    return true;
                }
                spec = false;
            }
        }
        return false;
    }
};

static int copy_out(const Bytes &b, uint8_t *out, int cap) {
    if ((int)b.size() > cap) return PXO_ESPACE;
    if (!b.empty()) memcpy(out, b.data(), b.size());
    return (int)b.size();
}

extern "C" {

pxo_shard *pxo_new(void) { return new pxo_shard(); }
void pxo_free(pxo_shard *s) { delete s; }

int pxo_set(pxo_shard *s, const uint8_t *k, int klen, const uint8_t *v, int vlen,
            uint32_t *chunk_no, uint32_t *idx) {
    try {
        Bytes doc;
        int rc = assemble_doc(k, klen, v, vlen, doc);
        if (rc) return rc;
        uint32_t c, i;
        rc = s->ctrl_set(doc, false, &c, &i);
        if (chunk_no) *chunk_no = c;
        if (idx) *idx = i;
        return rc;
    } catch (const Fail &f) {
        return f.code;
    }
}

// PiXiuCtrl::reinsert(PiXiuChunk *&) called directly (PiXiuCtrl.cpp:88-114) on closed chunk c:
// PXO_EINVAL for the live chunk or an unknown one
int pxo_reinsert(pxo_shard *s, uint32_t c) {
    if ((size_t)c + 1 >= s->chunks.size()) return PXO_EINVAL;
    try {
        s->reinsert_chunk((int)c, false);
    } catch (const Fail &f) {
        return f.code;
    }
    return 0;
}

int pxo_contains(pxo_shard *s, const uint8_t *k, int klen) {
    try {
        Bytes key;
        escape_append(k, klen, true, key);
        return s->contains(key) ? 1 : 0;
    } catch (const Fail &f) {
        return f.code;
    }
}

int pxo_delete(pxo_shard *s, const uint8_t *k, int klen) {
    try {
        Bytes key;
        escape_append(k, klen, true, key);
        s->delete_trigger();
        return s->remove(key);
    } catch (const Fail &f) {
        return f.code;
    }
}

int pxo_comp(pxo_shard *s, uint32_t chunk, uint32_t idx, uint8_t *out, int cap) {
    if (chunk >= s->chunks.size() || idx >= s->chunks[chunk].recs.size()) return PXO_EINVAL;
    return copy_out(s->chunks[chunk].recs[idx], out, cap);
}

int pxo_parse(pxo_shard *s, uint32_t chunk, uint32_t idx, int from, int to, int mode,
              uint8_t *out, int cap) {
    try {
        if (chunk >= s->chunks.size() || idx >= s->chunks[chunk].recs.size()) return PXO_EINVAL;
        if (from < 0 || to < from) return PXO_EINVAL;
        Sink sk;
        s->decode_into(chunk, idx, from, to, mode, sk);
        return copy_out(sk.out, out, cap);
    } catch (const Fail &f) {
        return f.code;
    }
}

int pxo_get(pxo_shard *s, const uint8_t *k, int klen, int mode, uint8_t *out, int cap) {
    try {
        Bytes key;
        escape_append(k, klen, true, key);
        Leaf l;
        if (!s->lookup(key, &l)) return PXO_NOTFOUND;
        Sink sk;
        s->decode_into(l.chunk, l.idx, 0, kMaxDoc, mode, sk);
        return copy_out(sk.out, out, cap);
    } catch (const Fail &f) {
        return f.code;
    }
}

// CritBitTree::find_best_match + key_eq (CritBitTree.cpp:185-195): where the key's
// record lives (chunk number, slot), for state comparisons after reinsert.
int pxo_locate(pxo_shard *s, const uint8_t *k, int klen, uint32_t *chunk, uint32_t *idx) {
    try {
        Bytes key;
        escape_append(k, klen, true, key);
        Leaf l;
        if (!s->lookup(key, &l)) return PXO_NOTFOUND;
        *chunk = l.chunk;
        *idx = l.idx;
        return 0;
    } catch (const Fail &f) {
        return f.code;
    }
}

// PiXiuCtrl::iter (PiXiuCtrl.cpp:71-75): the records yielded, in order.  Returns the
// count (-5 = PXO_NOTFOUND for an empty tree, the reference's NULL generator).
int pxo_iter(pxo_shard *s, const uint8_t *prefix, int plen, uint32_t *chunk_out, uint32_t *idx_out, int cap) {
    try {
        Bytes p;
        escape_append(prefix, plen, false, p);
        std::vector<Leaf> got;
        if (!s->iter(p, got)) return PXO_NOTFOUND;
        if ((int)got.size() > cap) return PXO_ESPACE;
        for (size_t i = 0; i < got.size(); ++i) {
            chunk_out[i] = got[i].chunk;
            idx_out[i] = got[i].idx;
        }
        return (int)got.size();
    } catch (const Fail &f) {
        return f.code;
    }
}

// Decode against a caller-supplied chunk of compressed records (decoder KATs).
int pxo_decode_chunk(int n, const uint8_t *comp, const uint64_t *off, int idx, int from, int to, int mode,
                     uint8_t *out, int cap) {
    try {
        Chunk ch;
        for (int i = 0; i < n; ++i) ch.recs.emplace_back(comp + off[i], comp + off[i + 1]);
        ch.dead.assign((size_t)n, 0);
        if (idx < 0 || idx >= n || from < 0 || to < from) return PXO_EINVAL;
        Sink sk;
        if (mode == PXO_COMPAT) {
            compat_parse(ch, (uint32_t)idx, from, to, sk, (size_t)-1, 0);
        } else {
            const Bytes &e = exact_expand(ch, (uint32_t)idx, 0);
            size_t a = std::min((size_t)from, e.size()), b = std::min((size_t)to, e.size());
            sk.out.assign(e.begin() + a, e.begin() + b);
        }
        return copy_out(sk.out, out, cap);
    } catch (const Fail &f) {
        return f.code;
    }
}

int pxo_last_fail_line(void) { return g_fail_line; }
int pxo_trace_take(int *out, int cap) {
    g_trace_on = true;
    int n = (int)g_trace.size();
    if (n > cap) return -1;
    for (int i = 0; i < n; ++i) out[i] = g_trace[(size_t)i];
    g_trace.clear();
    return n / 3;
}
int pxo_dump_tree(pxo_shard *s, char *out, int cap) {
    std::string t;
    s->gst.dump(0, 0, t);
    if ((int)t.size() + 1 > cap) return -1;
    memcpy(out, t.c_str(), t.size() + 1);
    return (int)t.size();
}
long pxo_ub_reads(pxo_shard *s) { return s->gst.ub_reads(); }
uint32_t pxo_num_chunks(pxo_shard *s) { return (uint32_t)s->chunks.size(); }
uint32_t pxo_chunk_records(pxo_shard *s, uint32_t chunk) {
    return chunk < s->chunks.size() ? (uint32_t)s->chunks[chunk].recs.size() : 0;
}
void pxo_pool_state(pxo_shard *s, int *pools, int *used_blocks) {
    if (pools) *pools = s->gst.pools();
    if (used_blocks) *used_blocks = s->gst.used_blocks();
}

int pxo_escape(const uint8_t *src, int n, int is_key, uint8_t *out, int cap) {
    Bytes b;
    escape_append(src, n, is_key != 0, b);
    return copy_out(b, out, cap);
}

int pxo_stream(int n, const int *cmd, const int *pos, const uint8_t *val, uint8_t *out, int cap) {
    StreamEncoder enc;
    Bytes res;
    enc.feed(Msg{kCmdOn, 0, 0}, nullptr);
    for (int i = 0; i < n; ++i) enc.feed(Msg{cmd[i], pos[i], val[i]}, nullptr);
    if (!enc.feed(Msg{kCmdOff, 0, 0}, &res)) return PXO_ECORRUPT;
    return copy_out(res, out, cap);
}

int pxo_run(int n, const uint8_t *keys, const uint64_t *koff, const uint32_t *klen,
            const uint8_t *vals, const uint64_t *voff, const uint32_t *vlen,
            uint8_t *comp, uint64_t comp_cap, uint64_t *comp_off,
            uint32_t *chunk_no, uint32_t *idx,
            int do_get, int mode, uint8_t *dec, uint64_t dec_cap, uint64_t *dec_off) {
    pxo_shard s;
    uint64_t c = 0;
    comp_off[0] = 0;
    for (int i = 0; i < n; ++i) {
        int rc = pxo_set(&s, keys + koff[i], (int)klen[i], vals + voff[i], (int)vlen[i], &chunk_no[i], &idx[i]);
        if (rc < 0) return rc;
        const Bytes &b = s.chunks[chunk_no[i]].recs[idx[i]];
        if (c + b.size() > comp_cap) return PXO_ESPACE;
        if (!b.empty()) memcpy(comp + c, b.data(), b.size());
        c += b.size();
        comp_off[i + 1] = c;
    }
    if (do_get) {
        uint64_t d = 0;
        dec_off[0] = 0;
        for (int i = 0; i < n; ++i) {
            uint64_t room = dec_cap - d;
            int m = pxo_get(&s, keys + koff[i], (int)klen[i], mode, dec + d,
                            (int)(room < 0x7fffffffu ? room : 0x7fffffffu));
            if (m == PXO_NOTFOUND) m = 0;
            if (m < 0) return m;
            d += (uint64_t)m;
            dec_off[i + 1] = d;
        }
    }
    return 0;
}

int pxo_encode_docs(int n, const uint8_t *docs, const uint64_t *doc_off,
                    uint8_t *comp, uint64_t comp_cap, uint64_t *comp_off,
                    uint32_t *chunk_no, uint32_t *idx) {
    try {
        pxo_shard s;
        uint64_t c = 0;
        comp_off[0] = 0;
        for (int i = 0; i < n; ++i) {
            Bytes doc(docs + doc_off[i], docs + doc_off[i + 1]);
            if (doc.size() > (size_t)kMaxDoc) return PXO_EINVAL;
            s.store(doc, &chunk_no[i], &idx[i]);
            const Bytes &b = s.chunks[chunk_no[i]].recs[idx[i]];
            if (c + b.size() > comp_cap) return PXO_ESPACE;
            if (!b.empty()) memcpy(comp + c, b.data(), b.size());
            c += b.size();
            comp_off[i + 1] = c;
        }
        return 0;
    } catch (const Fail &f) {
        return f.code;
    }
}

// MemPool state (pools, used blocks) after every doc, docs stored one after another as
// the single-instance reference does (rotation included): chunk_no[i] / pools[i] /
// used[i] after doc i.  Checks the suffix-array path's pool emulation (px_psa.hip).
int pxo_pool_trace(int n, const uint8_t *docs, const uint64_t *doc_off, uint32_t *chunk_no, int32_t *pools,
                   int32_t *used) {
    try {
        pxo_shard s;
        for (int i = 0; i < n; ++i) {
            Bytes doc(docs + doc_off[i], docs + doc_off[i + 1]);
            if (doc.size() > (size_t)kMaxDoc) return PXO_EINVAL;
            uint32_t idx = 0;
            s.store(doc, &chunk_no[i], &idx);
            pools[i] = s.gst.pools();
            used[i] = s.gst.used_blocks();
        }
        return 0;
    } catch (const Fail &f) {
        return f.code;
    }
}

}  // extern "C"
