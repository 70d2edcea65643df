// px_common.h — layouts shared by the HIP kernels (px_kernels.hip) and the host
// runtime (px_runtime.cpp).  Everything here is plain data: sizes and field order
// are part of the device ABI between the two translation units.
#pragma once
#include <stdint.h>

namespace px {

// ---- PiXiu encoding constants (PiXiuStr.h:11-21) ----
constexpr uint8_t kEsc = 251;      // PXS_UNIQUE
constexpr uint8_t kKeyEnd = 0;     // PXS_KEY
constexpr uint8_t kValEnd = 2;     // PXS_KEY_SEC
constexpr uint8_t kBigSign = 1;    // PXS_COMPRESS
constexpr int kMaxDoc = 65535;     // PXSG_MAX_TO
constexpr int kChunkSlots = 65535; // PXC_STR_NUM

// ---- MemPool emulation (MemPool.h:6-7, MemPool.cpp:7-37; PiXiuCtrl.cpp:13) ----
constexpr int kPoolBlocks = 65535;
constexpr int kNodeBlocks = 5;   // sizeof(STNode) = 40 B
constexpr int kEdgeBlocks = 3;   // sizeof(SGTNode<STNode>) = 24 B
constexpr int kRotatePools = 2048;

// ---- GST arena ----
// A node is just its suffix link (u32).  Every edge lives in its parent's child
// map as a 16-byte entry that carries the child's label, so one probe yields the
// child's id AND label (no second dependent load):
//   x = parent:26 | epoch:4 << 26      (epoch 0 == empty; rotation bumps the epoch)
//   y = child:26  | kids:1 << 26       (kids: the child has >= 1 child itself)
//   z = doc | from << 16               (label in the chunk-local doc `doc`)
//   w = to  | byte << 16               (byte = the key, the label's first byte)
// The root's 256 entries live in a direct table (LDS while a kernel runs).
// Non-root entries: open addressing over 64-byte buckets of 4 entries.
constexpr uint32_t kRoot = 0;
constexpr uint32_t kNone = 0xffffffffu;
constexpr int kNodeBits = 26;
constexpr uint32_t kNodeMask = (1u << kNodeBits) - 1;
constexpr uint32_t kMaxNodes = kNodeMask;
constexpr uint32_t kKidsBit = 1u << 26;
constexpr int kMaxEpoch = 15;
constexpr int kBucket = 4;  // entries per 64-byte bucket

// persistent per-shard GST state (device resident between batches)
struct ShardState {
    uint32_t n_nodes;      // nodes allocated in the live chunk (root included)
    int32_t pools;         // MemPool::nth
    int32_t used_blocks;   // MemPool::used_num
    int32_t pool_open;     // MemPool::curr_pool != NULL
    uint32_t n_docs;       // docs in the live chunk (SuffixTree::local_chunk.used_num)
    uint32_t chunk_seq;    // how many rotations this shard has seen
    uint32_t epoch;        // current hash epoch (1..15)
    uint32_t status;       // 0 ok, else a px_status (sticky: the shard is dead)
    uint64_t ctext_off;    // byte offset of the live chunk's text inside the arena text section
    uint64_t ub_reads;     // out-of-bounds reads the reference would make (UB there)
};

static_assert(sizeof(ShardState) % 16 == 0, "ShardState is zeroed / copied as 16-byte vectors");

// per-batch shard work descriptor
struct GstShard {
    uint8_t *text;        // arena text section
    uint32_t *doc_base;   // [doc_cap + 1] doc start relative to the live chunk text base
    uint4 *nodes;         // [2 * node_cap] node records (link, child count, two inline children)
    uint4 *hash;          // [hash_mask + 1] child-map entries
    uint4 *root;          // [256] root entries (y == kNone: absent)
    ShardState *st;
    uint32_t node_cap;
    uint32_t hash_mask;   // entries - 1 (a multiple of kBucket minus 1)
    uint32_t doc_cap;
    uint32_t r0, r1;      // batch records [r0, r1) belong to this shard, in order
    uint32_t replay;      // docs of the live chunk to re-walk first (tree not materialised)
};

// ---- PSA: the parallel suffix-array formulation of the GST walk (px_psa.hip,
// DESIGN.md §9).  A PSA shard's live chunk (earlier docs + this batch's) is one text
// in a global position space; every doc of it is listed, earlier docs with msg null.
struct PsaDoc {
    const uint8_t *src;  // escaped doc (in its shard's arena text)
    uint32_t *msg;       // its encoder messages, one u32 per byte (null: an earlier doc)
    uint32_t start;      // global position of its first byte
    uint32_t len;
    uint32_t shard;      // PSA shard index
    uint32_t slot;       // chunk-local idx (what reference tokens carry)
    uint32_t rec;        // batch record index (earlier docs: unused)
    uint32_t pad;
};
static_assert(sizeof(PsaDoc) == 40, "PsaDoc layout");
struct PsaShard {
    uint32_t base, len;  // global positions [base, base + len): also its suffix-array range
    uint32_t chunk;      // chunk sequence number of the live chunk
    uint32_t pools;      // 1: emulate MemPool (the live chunk can rotate inside this window)
    uint32_t doc0, ndocs;  // its docs in the PsaDoc list (the live chunk's, then the new ones)
    uint32_t pad[2];
};
static_assert(sizeof(PsaShard) == 32, "PsaShard layout");
// MemPool emulation result per PSA shard: the first doc (PsaDoc index) that goes to the
// next chunk (kNone: every doc stays), and the pool state after the last doc that stays
struct PsaPoolOut {
    uint32_t rot_doc;
    int32_t pools, used;  // (after the docs that stay; the bound test leaves them 0 / 2,048)
    uint32_t how;         // 0: the boundary chain ran, 1: the bound test (no rotation), 2: (rotation),
                          // 3: the chain stalled (no verdict: the shard goes to the walk)
};
// device scratch for px_psa.hip, borrowed from the runtime's heap
struct PsaAlloc {
    void *(*alloc)(void *self, uint64_t n);
    void (*release)(void *self, void *p, uint64_t n);
    void *self;
    uint32_t *pin;  // >= kPsaPinWords pinned host words (counts come back through them)
};
constexpr uint32_t kPsaPinWords = 512;
struct PsaStats {
    uint32_t iterations;  // prefix-doubling steps after the first sort
    uint32_t active[24];  // unsorted suffixes entering each doubling step
    float ms_sort, ms_lcp, ms_msg, ms_pool;
    uint32_t candidates;  // split candidates of the MemPool emulation
};
// a live chunk of at most this many doc bytes cannot rotate by pool count: MemPool charges
// <= 16 blocks per inserted leaf (leaf 5 + entry 3, split node 5 + entry 3) and at most one
// leaf per byte, a closed pool holds >= 65,531 blocks, and rotation needs 2,048 pools
// (PiXiuCtrl.cpp:13; MemPool.cpp:7-37): (2047 * 65531 - 5) / 16
constexpr uint32_t kPsaMaxText = (uint32_t)((2047ull * 65531ull - 5ull) / 16ull);
// device scratch per text position of one suffix-array round at its peak (px_psa.hip:
// text, doc ids, distances, ranks, suffix array, sort keys and values, flags, links, lcp,
// and the MemPool emulation's link records and candidate table), rounded up
constexpr uint64_t kPsaBytesPerPos = 96;
// shards per round: the first sort key holds the shard id in its top bits
constexpr uint32_t kPsaShardBits = 19;
constexpr uint32_t kPsaMaxShards = 1u << kPsaShardBits;

// segment index entry (k_tokenize / k_tok_segs fill it).  (Through round 5 it carried a
// second 16-byte half with an address per entry -- a plain segment's first byte, a record
// token's target entry -- that k_link wrote and no kernel read: the lane entries below carry
// the relative form the decoder uses.)
struct alignas(16) SegEnt {
    uint32_t x, ex;  // source range [x, ex) of the segment
    uint32_t kz;     // comp offset | kind << 30: 0 plain, 1 skip, 2 record, 3 end (sentinel)
    uint32_t aux;    // record token: idx | from << 16 (its to = from + ex - x)
};
static_assert(sizeof(SegEnt) == 16, "SegEnt is one 16-byte vector");

// lane-walk entry (k_decode's lanes), parallel to SegEnt k of the same record: one
// 16-byte load per step.  Only records whose source coordinates fit 16 bits (every
// record the encoder produces) have them; the serial path and the position lookups
// keep using SegEnt.
//   xe  = x | ex << 16
//   kz  = comp offset | kind << 30 (as SegEnt)
//   aux = record token: idx | from << 16
//   rel = plain: (the record's comp base - this entry's address) / 8 (same allocation);
//         record token: (target entry - this entry) / 16, kRelNone when unlinked or
//         too far away (the token then goes to the serial path)
struct alignas(16) LaneEnt {
    uint32_t xe, kz, aux;
    int32_t rel;
};
static_assert(sizeof(LaneEnt) == 16, "LaneEnt is one 16-byte vector");
constexpr int32_t kRelNone = (int32_t)0x80000000;

// a record token as k_gst_emit wrote it: k_tok_segs builds the record's segment index from its
// tokens (the plain segments lie between them) instead of parsing the compressed bytes again
struct alignas(16) TokEnt {
    uint32_t x;   // doc position of the run the token stands for (its source position)
    uint32_t o;   // comp offset of the token
    uint32_t w;   // idx | from << 16 (SegEnt::aux)
    uint32_t rs;  // run length | token bytes << 16
};
constexpr uint32_t kTokBad = 1u << 31;  // a record's token count flag: parse its bytes (k_tokenize) instead

// compressed-record slot: what a chunk table entry points at
struct alignas(16) RecSlot {
    const uint8_t *comp;    // compressed bytes
    const SegEnt *seg;      // segment index, nseg entries + an end sentinel (see k_tokenize)
    const uint16_t *pidx;   // position index: pidx[b] = segment holding source position 16b
    uint32_t comp_len;
    uint32_t nseg;
    uint32_t pidx_n;        // blocks in pidx (0: no position index, serial decode only)
    uint32_t seg_cap;       // segment entries the index has room for, sentinel included (0: sized by
                            // seg_entries of its 251 bytes); k_tokenize fails a record that needs more
    const LaneEnt *lane;    // lane-walk entries (null: serial decode only); 48 bytes in all
};
static_assert(sizeof(RecSlot) == 48, "RecSlot is loaded as three 16-byte vectors");

// k_shard_init work item: a brand-new shard arena (zeroed child map and state)
struct ShardInit {
    uint4 *hash;
    ShardState *st;
    uint64_t entries;
};

// k_scatter_slots work item: one new chunk-table entry
struct SlotPut {
    RecSlot *dst;
    RecSlot val;
};
// a set batch's record r: where its slot goes in its chunk's device table (null: not
// placed), its slot number and the chunk's record count (k_slot_place)
struct SlotDst {
    RecSlot *dst;
    uint32_t idx, nrec;
};

// k_link work item: one record whose record tokens get their target entries
struct LinkJob {
    SegEnt *seg;
    LaneEnt *lane;         // the record's lane entries (null: none)
    const RecSlot *slots;  // the record's chunk table
    uint32_t nseg, nrec;
};

// decode query
struct DecodeQuery {
    uint32_t chunk;       // global chunk id
    uint32_t idx;         // chunk-local record slot
    int32_t from, to;     // PiXiuStr::parse(from, to)
    uint64_t out_off;     // where the output goes
    uint32_t out_cap;     // consumer stops pulling after this many bytes
    uint32_t mode;        // 0 compat, 1 exact
    uint32_t nrec;        // records in the chunk (record tokens are bounds-checked against it)
    uint32_t pad;         // compat: the top frame's ret cursor at `from` (a piece of a whole drain), else 0
};

// Span table (fast full-range getitem): a record's compat expansion
// as literal runs of compressed bytes.  Entry k covers output [start_k, start_{k+1})
// and copies it from (the record's comp pointer + rel); a sentinel entry {0, len}
// closes the table.
struct SpanEnt {
    int32_t rel;
    uint32_t start;
};
constexpr int32_t kAddrNone = (int32_t)0x80000000;  // a source beyond +-2 GiB of the record
// k_decode_addr writes a run's address at its first output byte only; the array starts filled
// with kAddrMark (the byte continues the run before it: its address is the previous one + 1)
constexpr int32_t kAddrMark = (int32_t)0x80000001;

// span build work item: the address decode of one record (k_decode_addr's output), in one
// piece (addr, len) or in the pieces first..last of a piece table (pq[k].out_off, pl[k])
struct SpanJob {
    const int32_t *addr;  // per output run: source address relative to the record's comp (kAddrMark between)
    const uint8_t *base;  // the record's comp pointer
    const uint8_t *doc;   // the escaped doc (compat == exact test), or null
    SpanEnt *out;         // span entries (count pass: null)
    uint32_t len;         // output bytes (k_decode_addr's length)
    uint32_t doc_len;
    uint32_t *count;      // count pass: spans | kSpanBad, eq flag in bit 30
    uint32_t *tix;        // write pass: tile index (kGatherTile bytes per tile), or null
    const DecodeQuery *pq;  // pieces (null: one piece at addr)
    const uint32_t *pl;
    uint32_t first, last;
};
// span build source of one record: its escaped doc on the device (compat == exact test) or null
struct SpanSrc {
    const uint8_t *doc;
    uint32_t doc_len, pad;
};
// the gather's tile: one lane assembles kGatherTile output bytes; tix[t] = the span
// holding output byte t * kGatherTile
constexpr uint32_t kGatherTile = 32;
constexpr uint32_t kSpanBad = 1u << 31, kSpanEq = 1u << 30;

// gather query: one full-range getitem served from a span table
struct GatherQuery {
    const SpanEnt *span;
    const uint8_t *base;
    uint64_t out_off;
    uint32_t nspan, len, cap;
    uint32_t slot;    // result index (out_len / status)
    const uint32_t *tix;  // tile index of the span table
    uint32_t tile0;   // the launch's global tile number of this query's first tile
    uint32_t pad;
};

// ---- device key index (px_keyidx.hip): getitem's key -> record resolution on the GPU for
// the keys the host's own fast path would answer (px_runtime.cpp resolve_key: the newest
// record stored under the raw key, live, whose compat key prefix is the escaped key)
struct DkRec {
    const SpanEnt *sp;   // compat span table (null: none)
    const uint32_t *t;
    const SpanEnt *xsp;  // exact span table (null: none; == sp when the expansions agree)
    const uint32_t *xt;
    const uint8_t *comp;  // the record's compressed bytes
    uint64_t key_off;     // its raw key in the index's key arena
    uint32_t key_len, n, len, xn, xlen, doc_len, flags, pad;
};
static_assert(sizeof(DkRec) == 80, "DkRec layout");
constexpr uint32_t kDkLive = 1, kDkClean = 2;
struct DkSlot {
    unsigned long long h;  // key hash | 1; 0: empty
    uint32_t gid1;         // newest record id + 1 stored under the key
    uint32_t pad;
};

// gather task (64 tiles): the first query, the span holding the task's first tile in its
// table, and a bit per tile where a later query starts
struct alignas(16) GatherTask {
    uint32_t q0, k0;
    unsigned long long M;
};

// decode frame (scratch, one stack per wave)
struct alignas(16) Frame {
    uint32_t rec;     // chunk-local idx of the record being parsed ("self")
    int32_t from;
    int32_t len;
    int32_t ret;      // ret_cursor (relative, the reference's accounting)
    int32_t src;      // src_cursor (absolute within self)
    uint32_t seg;     // next segment to visit
    uint32_t cap;     // absolute output position where this frame's consumer stops
    uint32_t state;   // 0 run, 1 waiting on a plain child, 2 waiting on a periodic child
    uint32_t pstart;  // output position where the pending child began
    int32_t sub_from, sub_to, supply;
};
static_assert(sizeof(Frame) == 48, "Frame is moved as three 16-byte vectors");

enum Status : uint32_t {
    kOk = 0,
    kErrInval = 1,      // bad argument / oversize doc / empty key
    kErrCapacity = 2,   // arena too small (host sizing bug)
    kErrRefCrash = 3,   // reference would dereference NULL here (SuffixTree.cpp child lookup)
    kErrCorrupt = 4,    // malformed compressed bytes
    kErrHang = 5,       // reference decoder would loop forever
    kErrDepth = 6,      // decode stack exhausted
    kErrSpace = 7,      // output capacity exceeded (result truncated)
};

}  // namespace px
