// px_runtime.cpp — host runtime behind the C ABI (include/pixiu_amd.h).
//
// Owns device memory (a slab heap), the per-shard GST arenas, the compressed
// record store (chunk slot tables the decoder indexes), and the host-side
// CritBit index (the north star keeps it on the host).  Every data-path byte is
// produced by the HIP kernels in px_kernels.hip; the host only moves metadata
// (lengths, statuses, key prefixes) and runs the CritBit walk.
#include <hip/hip_runtime.h>
#include <malloc.h>
#include <array>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/pixiu_amd.h"
#include "px_common.h"
#include "px_host.h"
#include "px_sort.h"

namespace px {
hipError_t launch_doc_len(hipStream_t, uint32_t, const uint8_t *, const uint64_t *, const uint8_t *,
                          const uint64_t *, uint32_t *, uint32_t *);
hipError_t launch_doc_write(hipStream_t, uint32_t, const uint8_t *, const uint64_t *, const uint8_t *,
                            const uint64_t *, uint8_t *const *);
hipError_t launch_shard_init(hipStream_t, uint32_t, const ShardInit *);
hipError_t launch_scatter_slots(hipStream_t, uint32_t, const SlotPut *);
hipError_t launch_gst_encode(hipStream_t, const GstShard *, uint32_t, const uint32_t *, uint8_t *const *,
                             const uint8_t *, uint32_t *, uint32_t *, uint32_t *, uint32_t *, ShardState *,
                             uint32_t *);
hipError_t psa_run(hipStream_t, const PsaAlloc &, uint32_t, const PsaDoc *, uint32_t, const PsaShard *, const PsaShard *,
                   uint32_t,
                   uint32_t *, uint32_t *, uint32_t *, uint32_t *, bool, PsaPoolOut *, PsaStats *);
hipError_t launch_gst_emit(hipStream_t, uint32_t, const uint8_t *const *, const uint32_t *, uint8_t *const *,
                           const uint8_t *, const uint32_t *, uint32_t *, uint32_t *, const uint64_t *, TokEnt *, uint32_t *);
hipError_t launch_compact(hipStream_t, uint32_t, uint8_t *const *, const uint32_t *, uint8_t *, const uint64_t *);
hipError_t launch_tokenize(hipStream_t, uint32_t, const RecSlot *, uint32_t *, uint32_t *, const uint32_t *);
hipError_t launch_tok_segs(hipStream_t, uint32_t, const RecSlot *, const uint32_t *, const uint64_t *, const TokEnt *,
                           uint32_t *, uint32_t *, uint32_t *);
hipError_t launch_count_esc(hipStream_t, uint32_t, uint8_t *const *, const uint32_t *, uint32_t *);
hipError_t launch_link(hipStream_t, uint32_t, const LinkJob *);
hipError_t launch_decode(hipStream_t, const DecodeQuery *, uint32_t, const RecSlot *const *, uint8_t *,
                         uint32_t *, uint32_t *, Frame *, uint32_t, uint32_t, bool);
hipError_t launch_rehash(hipStream_t, const uint4 *, uint32_t, uint32_t, uint4 *, uint32_t);
hipError_t launch_decode_addr(hipStream_t, const DecodeQuery *, uint32_t, const RecSlot *const *, int32_t *,
                              uint32_t *, uint32_t *, Frame *, uint32_t, uint32_t);
hipError_t launch_slot_place(hipStream_t, uint32_t, const RecSlot *, const uint32_t *, const SlotDst *, LinkJob *);
hipError_t launch_span_agg(hipStream_t, uint32_t, const uint32_t *, const uint32_t *, const uint32_t *,
                           const DecodeQuery *, uint32_t *, uint32_t *);
hipError_t launch_span_pieces(hipStream_t, uint32_t, DecodeQuery *, const RecSlot *const *, uint32_t);
hipError_t launch_span_jobs(hipStream_t, uint32_t, const DecodeQuery *, const uint32_t *, const uint32_t *,
                            const SpanSrc *, const RecSlot *const *, const int32_t *, uint32_t *, uint32_t *,
                            uint32_t *, const uint32_t *, const uint32_t *, SpanEnt *, uint32_t *, const DecodeQuery *,
                            const uint32_t *, const uint32_t *);
uint64_t gather_task_bytes(uint32_t);
hipError_t launch_gather(hipStream_t, uint32_t, const uint32_t *, uint64_t, void *, const GatherQuery *, uint32_t,
                         uint8_t *, uint32_t *, uint32_t *);
hipError_t launch_dk_insert(hipStream_t, uint32_t, uint32_t, const DkRec *, const uint8_t *, DkSlot *, uint32_t,
                            uint32_t *);
hipError_t launch_dk_kill(hipStream_t, uint32_t, const uint32_t *, DkRec *);
hipError_t launch_dk_results(hipStream_t, uint32_t, const uint32_t *, uint64_t, const uint32_t *, const uint32_t *,
                             const uint32_t *, uint64_t *, uint32_t *, uint32_t *);
hipError_t launch_dk_lookup(hipStream_t, uint32_t, const uint8_t *, const uint64_t *, const DkSlot *, uint32_t,
                            const DkRec *, const uint8_t *, uint32_t, GatherQuery *, uint32_t *, uint32_t *,
                            unsigned long long *, const uint32_t *);
int debug_trace_take(int32_t *, uint32_t);
int debug_prof_take(unsigned long long *, uint32_t);
}  // namespace px

using namespace px;

namespace {

struct HipFail {
    hipError_t e;
    int line;  // px_runtime.cpp line of the failed call
};
inline void hcheck_at(hipError_t e, int line) {
    if (e != hipSuccess) throw HipFail{e, line};
}
#define hcheck(x) hcheck_at((x), __LINE__)
struct PxFail {
    int code;
};

inline uint64_t round_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }
// the fault-injecting test hooks (PX_DEBUG_SET_THROW, PX_DEBUG_FAIL_REC, PX_DEBUG_POISON) act
// only when PX_TEST_HOOKS=1 arms them as well, so a stray variable cannot break production
// batches
inline const char *test_hook(const char *name) {
    const char *armed = std::getenv("PX_TEST_HOOKS");
    if (!armed || armed[0] != '1') return nullptr;
    return std::getenv(name);
}
// position-index blocks for a record of `src_len` source bytes (k_tokenize)
inline uint32_t pidx_blocks(uint32_t src_len) { return src_len / 16 + 2; }
constexpr uint32_t kNoPidxBit = 1u << 31;  // k_tokenize: record has no position index
// segment entries for a compressed record holding `esc` 251 bytes: plain runs and
// tokens alternate, every token starts with a 251, plus the end sentinel
inline uint64_t seg_entries(uint32_t esc) { return 2ull * esc + 2; }
inline void set_nseg(RecSlot &s, uint32_t tok) {
    s.nseg = tok & ~kNoPidxBit;
    if (tok & kNoPidxBit) {
        s.pidx_n = 0;
        s.lane = nullptr;  // lane entries need monotone 16-bit source coordinates
    }
}
// set batches with more raw bytes than this (when one shard may take them all) are
// processed in pieces; a shard's live chunk text plus its batch must stay below
// kMaxShardText (32-bit text offsets through a 2^31-byte buffer resource)
constexpr uint64_t kMaxBatchRaw = 512ull << 20;
constexpr uint64_t kMaxShardText = (2ull << 30) - (64ull << 20);
// nodes a live chunk can hold: rotation happens before a doc once MemPool has opened
// 2,048 pools (PiXiuCtrl.cpp:13), so a doc starts with <= 2,047 x 65,535 blocks in use
// (a node costs 5 of them, MemPool.cpp:7-37) and adds at most 2 nodes per byte.
// Sizing node and hash sections from this bound (not from the batch bytes) keeps every
// arena offset below 2^31 (nodes 863 MB + hash 512 MB).
constexpr uint64_t kChunkNodeCap = (uint64_t)(kRotatePools - 1) * kPoolBlocks / kNodeBlocks + 2ull * kMaxDoc + 64;
static_assert(kChunkNodeCap <= kMaxNodes, "node ids are 26 bits");
inline uint64_t pow2_at_least(uint64_t v) {
    uint64_t p = 1024;
    while (p < v) p <<= 1;
    return p;
}

// ---------------------------------------------------------------- device heap
// px_host.h's best-fit block heap over 1 GiB hipMalloc slabs: batches of varying sizes
// reuse the same memory instead of growing the footprint; no hipMalloc per shard.
struct HipRaw {
    static void *get(uint64_t n) {
        void *v = nullptr;
        return hipMalloc(&v, n) == hipSuccess ? v : nullptr;
    }
    static void put(void *p) { (void)hipFree(p); }
};
class DevHeap : public pxh::BlockHeap<HipRaw> {
  public:
    void *alloc(uint64_t n) {
        void *p = BlockHeap::alloc(n);
        if (!p) throw PxFail{PX_ENOMEM};
        return p;
    }
    void release(void *v, uint64_t) { BlockHeap::release(v); }
};

// pinned-free scratch buffer that only grows
struct DevBuf {
    void *p = nullptr;
    uint64_t cap = 0;
    void *get(uint64_t n) {
        if (n > cap) {
            if (p) (void)hipFree(p);
            cap = std::max<uint64_t>(round_up(n, 1 << 20), cap * 2);
            p = nullptr;
            if (hipMalloc(&p, cap) != hipSuccess) {
                cap = 0;
                throw PxFail{PX_ENOMEM};
            }
        }
        return p;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// Record stores in one reserved virtual range, mapped on demand and allocated by a bump
// pointer (they are only ever freed together, at reset).  Span tables address a record's
// source bytes relative to the record itself with 32-bit offsets (SpanEnt::rel), so every
// record of a chunk has to lie within +-2 GiB of the others; separate heap allocations gave
// no such bound (a single instance's batch stored in two 512 MB pieces put one chunk's
// records in blocks further apart than that once the heap had been reused, and those
// records lost their span tables).  Appended in order, a chunk's records are as far apart
// as the bytes stored while the chunk was live.  Without virtual memory management the
// caller falls back to the heap.
struct StoreArena {
    char *base = nullptr;
    uint64_t reserved = 0, mapped = 0, top = 0, gran = 0;
    bool off = false;
    int device = 0;
    hipMemAllocationProp prop{};
    std::vector<std::pair<hipMemGenericAllocationHandle_t, uint64_t>> maps;  // in address order
    static constexpr uint64_t kReserve = 1ull << 40;                      // 1 TiB of addresses
    bool owns(const void *p) const { return base && (const char *)p >= base && (const char *)p < base + reserved; }
    void *alloc(uint64_t bytes) {
        if (off || std::getenv("PX_NO_STORE_ARENA")) return nullptr;
        if (!base) {
            int vmm = 0;
            if (hipGetDevice(&device) != hipSuccess ||
                hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, device) != hipSuccess || !vmm) {
                off = true;
                return nullptr;
            }
            prop.type = hipMemAllocationTypePinned;
            prop.location.type = hipMemLocationTypeDevice;
            prop.location.id = device;
            size_t g = 0;
            if (hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityRecommended) != hipSuccess || !g ||
                hipMemAddressReserve((void **)&base, kReserve, 0, nullptr, 0) != hipSuccess || !base) {
                base = nullptr;
                off = true;
                return nullptr;
            }
            gran = round_up(std::max<uint64_t>(g, 64ull << 20), g);  // (every mapping 64 MiB-aligned: the
                                                                    // minimum granularity let a second
                                                                    // mapping's access grant fail)
            reserved = kReserve;
        }
        static const bool verbose = std::getenv("PX_ARENA_VERBOSE") != nullptr;
        const uint64_t at = round_up(top, 256), end = at + bytes;
        if (verbose) fprintf(stderr, "arena: alloc %lu at %lu (mapped %lu)\n", (unsigned long)bytes, (unsigned long)at, (unsigned long)mapped);
        if (end > reserved) return nullptr;
        if (end > mapped) {  // map more: what is needed, at least 64 MiB and a quarter of what is mapped
            uint64_t want = std::max<uint64_t>(end - mapped, std::max<uint64_t>(64ull << 20, mapped / 4));
            want = round_up(want, gran);
            if (mapped + want > reserved) want = reserved - mapped;
            hipMemGenericAllocationHandle_t h{};
            hipError_t e = hipMemCreate(&h, want, &prop, 0);
            if (verbose) fprintf(stderr, "arena: create %lu -> %d\n", (unsigned long)want, (int)e);
            if (e != hipSuccess) {
                (void)hipGetLastError();  // (not sticky for the caller's next launch check)
                return nullptr;
            }
            e = hipMemMap(base + mapped, want, 0, h, 0);
            if (verbose) fprintf(stderr, "arena: map at %lu -> %d\n", (unsigned long)mapped, (int)e);
            if (e != hipSuccess) {
                (void)hipMemRelease(h);
                (void)hipGetLastError();
                return nullptr;
            }
            hipMemAccessDesc d{};
            d.location = prop.location;
            d.flags = hipMemAccessFlagsProtReadWrite;
            e = hipMemSetAccess(base + mapped, want, &d, 1);
            if (e != hipSuccess) {  // (ROCm grants access to a later mapping with the whole range)
                (void)hipGetLastError();
                e = hipMemSetAccess(base, mapped + want, &d, 1);
            }
            if (verbose) fprintf(stderr, "arena: access -> %d\n", (int)e);
            if (e != hipSuccess) {
                (void)hipMemUnmap(base + mapped, want);
                (void)hipMemRelease(h);
                (void)hipGetLastError();
                return nullptr;
            }
            maps.emplace_back(h, want);
            mapped += want;
        }
        top = end;
        return base + at;
    }
    // every block at once; the mapped memory stays for reuse (remapping an address range the
    // device has used was measured to leave copies and kernels reading the old pages: a store
    // reset and reloaded read back corrupt records)
    void reset() { top = 0; }
    ~StoreArena() {
        if (!base) return;
        (void)hipDeviceSynchronize();
        uint64_t o = 0;
        for (auto &m : maps) {
            (void)hipMemUnmap(base + o, m.second);
            (void)hipMemRelease(m.first);
            o += m.second;
        }
        (void)hipMemAddressFree(base, reserved);
    }
};

// pinned host staging buffer (grown on demand): small per-batch transfers without the
// runtime's pageable-copy path
struct HostBuf {
    void *p = nullptr;
    uint64_t cap = 0;
    void *get(uint64_t n) {
        if (n > cap) {
            if (p) (void)hipHostFree(p);
            cap = std::max<uint64_t>(round_up(n, 1 << 16), cap * 2);
            p = nullptr;
            if (hipHostMalloc(&p, cap, hipHostMallocDefault) != hipSuccess) {
                cap = 0;
                throw PxFail{PX_ENOMEM};
            }
        }
        return p;
    }
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
};

using pxh::KeyMap;
using pxh::parallel_ranges;
using pxh::PartKeyMap;
using pxh::PhaseClock;
using pxh::WorkerPool;

// ---------------------------------------------------------------- crit-bit index
// px_host.h's CritBit (CritBitTree.cpp:13-269 restated over the compat-decoded key
// prefixes of the stored records); one tree per shard.
using pxh::CbtInner;
using pxh::CbtRef;
using pxh::crit_dir;
using pxh::Leaf;
static_assert(pxh::kEscByte == kEsc && pxh::kKeyEndByte == kKeyEnd, "escape bytes");

struct Chunk {
    uint32_t shard = 0;
    uint32_t n = 0;
    uint32_t used = 0;   // PiXiuChunk::used_num: live records (placed, not deleted)
    uint32_t total = 0;  // PiXiuChunk::total_num: records when the chunk was closed (0: live)
    std::vector<RecSlot> slots;  // host mirror (device pointers inside)
    RecSlot *dev = nullptr;      // device slot table
    uint32_t dev_cap = 0;
    std::vector<uint32_t> doc_len;
    std::vector<uint8_t> dead;
    std::string kp;  // concatenated compat key prefixes
    std::vector<uint64_t> kp_off;
    std::vector<uint32_t> kp_len;
    std::vector<uint32_t> gid;  // device key index record id of each slot (kNone / past the end: none)
    // slots whose CritBit insert the reference skips (CritBitTree.cpp:96-100: the streams part
    // right after a 251): stored and live, but no walk reaches them (past the end: 0)
    std::vector<uint8_t> notree;
    bool in_tree(uint32_t i) const { return i >= notree.size() || !notree[i]; }
    // span tables (full-range getitem as a gather); sized lazily
    struct Span {
        const SpanEnt *p = nullptr;  // device; null: decode through the segment walk
        const uint32_t *t = nullptr;  // its tile index (the span at every kGatherTile-th byte)
        uint32_t n = 0, len = 0;     // spans, compat expansion length
        bool eq = false;             // the compat expansion equals the doc (== exact)
        const SpanEnt *xp = nullptr;  // exact expansion's table when it differs (!eq)
        const uint32_t *xt = nullptr;
        uint32_t xn = 0, xlen = 0;
    };
    std::vector<Span> span;
};

struct Shard : pxh::CritBit {
    uint32_t id = 0;
    // device arena
    void *arena = nullptr;
    uint64_t arena_bytes = 0;
    ShardState *st = nullptr;
    uint4 *root_tab = nullptr;
    uint32_t *doc_base = nullptr;
    uint4 *nodes = nullptr;
    uint4 *hash = nullptr;
    uint8_t *text = nullptr;
    uint32_t node_cap = 0, doc_cap = 0;
    uint64_t hash_cap = 0, text_cap = 0;
    ShardState hs{};      // host mirror after the last batch
    uint64_t text_end = 0;  // end of written text (relative to the arena text section)
    // the live chunk was encoded by the suffix-array path (px_psa.hip): hs.n_docs docs,
    // no tree; the arena is then text only (text_only) until a walk needs the tree
    bool psa = false, text_only = false;
    // Glob_Reinsert_Chunk of this shard's PiXiuCtrl (PiXiuStr.cpp:4, 178-187): the last
    // chunk a delete left under 80 % of 65,535 live records; -1 = NULL
    int64_t glob = -1;
    int64_t closed = -1;  // slot-full live chunk whose rotation trigger has run
    // a leaf went into this shard's CritBit under a key its compat-decoded prefix does not
    // equal: the trie is then only as consistent as the reference's, so every lookup walks it
    bool unclean = false;
    uint32_t records = 0;
    std::vector<uint32_t> chunks;  // global chunk ids by chunk_seq
};

}  // namespace

namespace {
px_status map_status(uint32_t s);  // device status -> px_status (defined below)
uint32_t key_end(const uint8_t *p, uint32_t n);  // (defined below)
}  // namespace

struct px_ctx {
    px_opts opts{};
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_mid = nullptr;
    hipEvent_t ev_get = nullptr;  // (a getitem batch's end: polled, not slept on)
    // wait for the stream by polling an event: a getitem batch's ~0.8 ms of kernels ended in a
    // blocking synchronize whose wake-up was a visible part of the call (PX_GET_SPIN=0: sleep)
    void spin_sync() {
        static const bool spin = [] {
            const char *e = std::getenv("PX_GET_SPIN");
            return !(e && e[0] == '0');
        }();
        if (!spin) {
            hcheck(hipStreamSynchronize(stream));
            return;
        }
        hcheck(hipEventRecord(ev_get, stream));
        for (;;) {
            const hipError_t q = hipEventQuery(ev_get);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) hcheck(q);
        }
    }
    hipStream_t stream2 = nullptr;  // getitem's second decode launch (get_overlapped)
    hipEvent_t ev_join = nullptr;
    DevHeap heap;
    std::vector<std::unique_ptr<Shard>> shards;
    std::vector<Chunk> chunks;
    RecSlot **chunk_tab = nullptr;  // device: chunk id -> slot table
    uint32_t chunk_tab_cap = 0;
    uint32_t tab_lo = ~0u, tab_hi = 0;      // chunk_tab entries not yet uploaded
    std::vector<ShardInit> pending_init;    // new shard arenas to zero (k_shard_init)
    std::vector<std::pair<ShardState *, ShardState>> pending_state;  // states set after the zeroing (loaded shards)
    PartKeyMap keymap;  // raw key -> shard (multi-shard only)
    std::vector<std::pair<void *, uint64_t>> store_blocks;  // packed record stores + segment indexes
    // stored-data bytes by structure (px_stats mem_*; only px_reset frees stored data)
    struct MemAcct {
        uint64_t comp = 0, lane = 0, seg = 0, pidx = 0, span = 0;
    } macct;
    StoreArena arena;                                        // (record stores: StoreArena above)
    void *store_alloc(uint64_t bytes) {
        if (void *p = arena.alloc(bytes)) return p;
        return heap.alloc(bytes);
    }
    uint8_t *last_store = nullptr;  // packed compressed bytes of the last set batch
    uint64_t last_store_bytes = 0;
    DevBuf scratch_frames, dq_buf, dstat_buf, dlen_buf, in_buf, tmp_buf, link_buf, iter_buf, init_buf, stout_buf,
        slotput_buf;
    HostBuf hq_buf, hres_buf;  // pinned: decode queries up, lengths + statuses down
    HostBuf hg_buf[2];         // pinned: gather queries up (a head and a tail launch)
    HostBuf psa_pin;
    HostBuf slot_pin;          // pinned: set_batch's slot entries on their way to the device
    HostBuf dst_pin;           // pinned: set_batch's doc and comp-scratch destinations
    HostBuf piece_pin;         // pinned: the span build's piece queries
    HostBuf src_pin;           // pinned: the span build's sources (doc pointers and lengths)           // pinned: px_psa.hip's count read-backs
    HostBuf kp_hbuf;           // pinned: decoded key prefixes down
    DevBuf sink_buf;           // k_gst_encode's message sink for replayed docs
    PsaStats psa_stats{};      // the last set batch's suffix-array pass
    // PX_PSA=0 sends every shard through k_gst_encode (A/B comparisons, tests)
    static bool psa_enabled() {
        const char *e = std::getenv("PX_PSA");
        return !(e && *e == '0');
    }
    // text positions one suffix-array round may take: its scratch (kPsaBytesPerPos per
    // position, px_psa.hip) must fit the free device memory, and positions are 32-bit.
    // PX_PSA_ROUND_MAX (positions) lowers it (tests of the multi-round path).
    uint64_t psa_round_cap() {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
        uint64_t cap = (uint64_t)(0.85 * (double)(fr + heap.cached_free())) / kPsaBytesPerPos;
        cap = std::min<uint64_t>(cap, 0x7ff00000ull);  // (group sizes carry a tag bit: < 2^31)
        if (const char *e = std::getenv("PX_PSA_ROUND_MAX")) cap = std::min<uint64_t>(cap, std::strtoull(e, nullptr, 10));
        return std::max<uint64_t>(cap, 1);
    }
    uint32_t host_threads() const {
        const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
        return opts.host_threads ? opts.host_threads : std::min(16u, hw);
    }
    px_stats stats{};
    int last_hip = 0;

    // ------------------------------------------------------------ write-behind queue
    // (opts.defer_bytes, records_per_shard == 0: the facade's one-record setitem calls).
    // Queued records are stored together by flush_queue(), before any other call on the
    // context and once defer_bytes raw bytes are pending.  The stored bytes equal those of
    // one call per record: chunk rotation and the reinsert triggers depend only on the
    // doc order, which the queue keeps, and set_ctrl evaluates the triggers between
    // records exactly as it does for a one-record call.
    std::vector<uint8_t> dq_k, dq_v;          // queued keys / values (host CSR)
    std::vector<uint64_t> dq_ko{0}, dq_vo{0};
    std::vector<uint32_t> dq_pred;            // `replaced` as returned at call time
    std::unordered_set<std::string> dq_keys;  // their escaped keys
    px_set_result last_res{};                 // the most recently stored record's result
    bool have_last = false;
    int dq_rc = PX_OK;                        // first failure among flushed records since px_flush
    bool defer_on() const { return opts.defer_bytes != 0 && opts.records_per_shard == 0; }
    int set_deferred(uint32_t n, const uint8_t *keys, const uint64_t *koff, const uint8_t *vals,
                     const uint64_t *voff, px_set_result *res);
    int flush_queue();
    void drop_queue() {
        dq_k.clear();
        dq_v.clear();
        dq_ko.assign(1, 0);
        dq_vo.assign(1, 0);
        dq_pred.clear();
        dq_keys.clear();
    }
    void note_last(uint32_t n, const px_set_result *res) {
        if (n && res) {
            last_res = res[n - 1];
            have_last = true;
        }
    }
    // ------------------------------------------------------------ device key index
    // (px_keyidx.hip): raw key -> newest record stored under it, on the device, so a
    // getitem batch whose every key the host's fast path would answer (resolve_key: that
    // record live and its compat key prefix the escaped key) resolves without host
    // lookups.  Any key it cannot answer sends the batch to the host path.
    struct Dki {
        bool valid = true;  // false after a mutation the index does not follow (px_load) until reset
        uint32_t nrec = 0;  // record ids handed out
        DkRec *rec = nullptr;
        uint64_t rec_cap = 0;
        uint8_t *keys = nullptr;
        uint64_t keys_len = 0, keys_cap = 0;
        DkSlot *tab = nullptr;
        uint32_t tab_cap = 0;     // slots, a power of two >= 2 x records
        uint32_t *err = nullptr;  // device word: an insert gave up (cannot happen)
        std::vector<uint32_t> kills;  // ids killed (replace / delete) since the last commit
        uint32_t miss_streak = 0, skipped = 0;  // getitem batches in a row the index could not answer
        uint32_t max_len = 0;  // the longest span-table expansion of any entry (bounds a batch's gather grid)
        std::mutex mu;
    } dki;
    static bool dki_enabled() {  // PX_DKI=0: every getitem resolves its keys on the host
        static const bool on = [] {
            const char *e = std::getenv("PX_DKI");
            return !(e && e[0] == '0');
        }();
        return on;
    }
    void dki_clear() {
        if (dki.rec) heap.release(dki.rec, dki.rec_cap * sizeof(DkRec));
        if (dki.keys) heap.release(dki.keys, dki.keys_cap);
        if (dki.tab) heap.release(dki.tab, (uint64_t)dki.tab_cap * sizeof(DkSlot));
        if (dki.err) heap.release(dki.err, 256);
        dki.rec = nullptr;
        dki.keys = nullptr;
        dki.tab = nullptr;
        dki.err = nullptr;
        dki.rec_cap = dki.keys_cap = dki.keys_len = 0;
        dki.tab_cap = dki.nrec = 0;
        dki.miss_streak = 0;
        dki.kills.clear();
        for (auto &c : chunks) c.gid.clear();
    }
    void dki_commit(uint32_t gid0, const DkRec *recs, uint32_t nn, const uint8_t *kb, uint64_t kbn);
    // a set batch's new index entries and their raw key bytes, in pinned memory kept across
    // batches: copied to the device straight from here (80 MB for a million records went
    // through the bulk ring's staging copy)
    HostBuf dk_rec_pin, dk_key_pin;
    // the live bit of every record killed since (replaces, deletes, reinsert), on the device
    void dki_apply_kills() {
        std::vector<uint32_t> kills;
        kills.swap(dki.kills);
        if (kills.empty() || !dki.rec) return;
        auto *d = (uint32_t *)dk_kbuf.get(kills.size() * 4);
        h2d(d, kills.data(), kills.size() * 4);
        hcheck(launch_dk_kill(stream, (uint32_t)kills.size(), d, dki.rec));
    }
    DevBuf dk_kbuf;
    // dev_io: keys, koff, out_off, out_len and status are device pointers (px_get_batch_dev)
    int dki_get(uint32_t n, const uint8_t *keys, const uint64_t *koff, int mode, uint8_t *out, uint64_t out_cap,
                int out_on_device, uint64_t *out_off, uint32_t *out_len, uint32_t *status, uint64_t *needed,
                bool dev_io = false);
    DevBuf dk_qbuf, dk_obuf;
    HostBuf dk_hbuf, dk_hres;

    // cached free device memory kept after a set batch (opts.retain_mb).  0 (the default):
    // what the batch itself needed at its peak beyond what stays live, so a workload of
    // similar batches never hands memory back to the driver and maps it again (round 4
    // freed ~25 GB after every config-3 batch and re-allocated it inside the next one);
    // memory beyond that (a batch larger than the ones after it) goes back.  The adaptive
    // amount is capped at half of what the device could give this process now (its free
    // memory plus what the heap caches), so other allocators in the process (torch's) keep
    // at least as much as the cache.  px_trim() returns cached memory on request.
    void trim_heap() {
        if (opts.retain_mb == 0xffffffffu) return;
        const uint64_t live = heap.live_bytes();
        uint64_t keep = opts.retain_mb ? (uint64_t)opts.retain_mb << 20 : heap.live_peak() - std::min(heap.live_peak(), live);
        if (!opts.retain_mb) {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess) keep = std::min<uint64_t>(keep, ((uint64_t)fr + heap.cached_free()) / 2);
        }
        heap.trim(keep);
    }

    // stored-data device bytes by structure (px_stats mem_*)
    void mem_stats(px_stats *st) const {
        st->mem_text_bytes = st->mem_tree_bytes = 0;
        for (const auto &sp : shards)
            if (sp->arena) (sp->text_only ? st->mem_text_bytes : st->mem_tree_bytes) += sp->arena_bytes;
        st->mem_comp_bytes = macct.comp;
        st->mem_lane_bytes = macct.lane;
        st->mem_seg_bytes = macct.seg;
        st->mem_pidx_bytes = macct.pidx;
        st->mem_span_bytes = macct.span;
        uint64_t sl = (uint64_t)chunk_tab_cap * sizeof(RecSlot *);
        for (const auto &c : chunks) sl += (uint64_t)c.dev_cap * sizeof(RecSlot);
        st->mem_slot_bytes = sl;
        st->mem_keyidx_bytes = dki.rec_cap * sizeof(DkRec) + dki.keys_cap + (uint64_t)dki.tab_cap * sizeof(DkSlot);
    }

    // ------------------------------------------------------------ helpers
    // Host->device copies are staged in buffers owned until the next sync(), so the
    // caller's (pageable, possibly short-lived) source may go away immediately.
    std::vector<std::vector<uint8_t>> staged;
    // Device->host copies never DMA into pageable memory: a small copy lands in pinned
    // staging (pre-filled with 0xff, so a copy that did not land reads as all-ones, not
    // as a plausible zero) and sync() moves it to its destination after the stream has
    // drained; a large one goes through a pinned bounce buffer synchronously.  Round 1
    // read result vectors filled by back-to-back pageable hipMemcpyAsync calls: once, a
    // record read status 0 / comp_len 0 -- the zero-initialised vector values, i.e. a
    // copy that had not landed.
    struct PendingD2H {
        void *dst;
        const void *src;
        size_t n;
    };
    std::vector<PendingD2H> pending_d2h;
    std::vector<std::pair<uint8_t *, size_t>> pin_blocks;  // pinned staging blocks (kept)
    size_t pin_blk = 0, pin_used = 0;
    static constexpr size_t kPinBlock = 4u << 20;
    uint8_t *pin_alloc(size_t n) {
        n = round_up(n, 64);
        while (pin_blk < pin_blocks.size() && pin_used + n > pin_blocks[pin_blk].second) {
            ++pin_blk;
            pin_used = 0;
        }
        if (pin_blk == pin_blocks.size()) {
            void *p = nullptr;
            const size_t sz = std::max(n, kPinBlock);
            if (hipHostMalloc(&p, sz, hipHostMallocDefault) != hipSuccess) throw PxFail{PX_ENOMEM};
            pin_blocks.emplace_back(static_cast<uint8_t *>(p), sz);
            pin_used = 0;
        }
        uint8_t *p = pin_blocks[pin_blk].first + pin_used;
        pin_used += n;
        return p;
    }
    void sync() {
        hcheck(hipStreamSynchronize(stream));
        for (const PendingD2H &c : pending_d2h) std::memcpy(c.dst, c.src, c.n);
        pending_d2h.clear();
        pin_blk = pin_used = 0;
        staged.clear();
    }
    void h2d(void *d, const void *h, size_t n) {
        if (!n) return;
        if (n >= kRingSlot) return h2d_bulk(d, h, n);  // large: pinned ring, no staging copy
        const uint8_t *b = static_cast<const uint8_t *>(h);
        staged.emplace_back(b, b + n);
        hcheck(hipMemcpyAsync(d, staged.back().data(), n, hipMemcpyHostToDevice, stream));
    }
    // Bulk host->device copies (the raw records of a host-buffer set batch): a ring of
    // pinned slots, the memcpy into one slot overlapping the DMA out of the others, so
    // the bytes cross PCIe once at pinned speed instead of through a pageable copy of
    // the whole batch. Returns once every byte has been copied out of the source.
    static constexpr size_t kRingSlot = 8u << 20;
    static constexpr int kRingSlots = 4;
    HostBuf ring_buf;
    hipEvent_t ring_ev[kRingSlots] = {};
    bool ring_busy[kRingSlots] = {};
    void h2d_bulk(void *d, const void *h, size_t n) {
        if (n < kRingSlot) {
            const uint8_t *b = static_cast<const uint8_t *>(h);
            staged.emplace_back(b, b + n);
            hcheck(hipMemcpyAsync(d, staged.back().data(), n, hipMemcpyHostToDevice, stream));
            return;
        }
        auto *slots = static_cast<uint8_t *>(ring_buf.get(kRingSlot * kRingSlots));
        const auto *src = static_cast<const uint8_t *>(h);
        auto *dst = static_cast<uint8_t *>(d);
        for (size_t o = 0, i = 0; o < n; o += kRingSlot, ++i) {
            const int k = (int)(i % kRingSlots);
            if (!ring_ev[k]) hcheck(hipEventCreateWithFlags(&ring_ev[k], hipEventDisableTiming));
            if (ring_busy[k]) hcheck(hipEventSynchronize(ring_ev[k]));
            const size_t m = std::min(kRingSlot, n - o);
            memcpy(slots + k * kRingSlot, src + o, m);
            hcheck(hipMemcpyAsync(dst + o, slots + k * kRingSlot, m, hipMemcpyHostToDevice, stream));
            hcheck(hipEventRecord(ring_ev[k], stream));
            ring_busy[k] = true;
        }
    }
    void d2h(void *h, const void *d, size_t n) {
        if (!n) return;
        // (async through kept pinned blocks up to 32 MB: a million-record batch reads back six
        // 4 MB arrays after its encode, which the synchronous bounce path took one by one)
        if (n <= (32u << 20)) {
            uint8_t *p = pin_alloc(n);
            std::memset(p, 0xff, n);
            hcheck(hipMemcpyAsync(p, d, n, hipMemcpyDeviceToHost, stream));
            pending_d2h.push_back(PendingD2H{h, p, n});
            return;
        }
        // large: through one pinned bounce block, piece by piece (synchronous)
        sync();
        uint8_t *bounce = pin_alloc(kPinBlock);
        auto *dst = static_cast<uint8_t *>(h);
        const auto *src = static_cast<const uint8_t *>(d);
        for (size_t o = 0; o < n; o += kPinBlock) {
            const size_t m = std::min(kPinBlock, n - o);
            hcheck(hipMemcpyAsync(bounce, src + o, m, hipMemcpyDeviceToHost, stream));
            hcheck(hipStreamSynchronize(stream));
            std::memcpy(dst + o, bounce, m);
        }
        pin_blk = pin_used = 0;
    }

    Shard &new_shard() {
        auto s = std::make_unique<Shard>();
        s->id = (uint32_t)shards.size();
        shards.push_back(std::move(s));
        stats.shards = shards.size();
        return *shards.back();
    }

    uint32_t new_chunk(uint32_t shard) {
        chunks.emplace_back();
        chunks.back().shard = shard;
        uint32_t id = (uint32_t)chunks.size() - 1;
        if (chunks.size() > chunk_tab_cap) {
            uint32_t cap = std::max<uint32_t>(1024, chunk_tab_cap * 2);
            while (cap < chunks.size()) cap *= 2;
            auto *nt = (RecSlot **)heap.alloc((uint64_t)cap * sizeof(RecSlot *));
            if (chunk_tab) {
                hcheck(hipMemcpyAsync(nt, chunk_tab, (size_t)chunk_tab_cap * sizeof(RecSlot *),
                                      hipMemcpyDeviceToDevice, stream));
                heap.release(chunk_tab, (uint64_t)chunk_tab_cap * sizeof(RecSlot *));
            }
            chunk_tab = nt;
            chunk_tab_cap = cap;
        }
        stats.chunks = chunks.size();
        return id;
    }

    // ensure chunk c's device slot table holds `need` slots
    void chunk_reserve(uint32_t c, uint32_t need) {
        Chunk &ch = chunks[c];
        if (need <= ch.dev_cap) return;
        uint32_t cap = std::max<uint32_t>(64, ch.dev_cap * 2);
        while (cap < need) cap *= 2;
        cap = std::min<uint32_t>(cap, kChunkSlots);
        auto *nt = (RecSlot *)heap.alloc((uint64_t)cap * sizeof(RecSlot));
        if (ch.dev) {
            // the old table's slots (new ones are scattered in afterwards; ch.n may already
            // count them, and reading past the old allocation is out of bounds)
            hcheck(hipMemcpyAsync(nt, ch.dev, (size_t)std::min(ch.n, ch.dev_cap) * sizeof(RecSlot),
                                  hipMemcpyDeviceToDevice, stream));
            heap.release(ch.dev, (uint64_t)ch.dev_cap * sizeof(RecSlot));
        }
        ch.dev = nt;
        ch.dev_cap = cap;
        tab_lo = std::min(tab_lo, c);
        tab_hi = std::max(tab_hi, c + 1);
    }

    // upload the chunk_tab entries changed since the last flush (one transfer)
    void flush_tab() {
        if (tab_lo >= tab_hi) return;
        std::vector<RecSlot *> v(tab_hi - tab_lo);
        for (uint32_t c = tab_lo; c < tab_hi; ++c) v[c - tab_lo] = chunks[c].dev;
        h2d(chunk_tab + tab_lo, v.data(), v.size() * sizeof(RecSlot *));
        tab_lo = ~0u;
        tab_hi = 0;
    }

    // zero the new shard arenas of this batch (one transfer + one launch)
    void flush_shard_init() {
        if (pending_init.empty()) return;
        auto *d = (ShardInit *)init_buf.get(pending_init.size() * sizeof(ShardInit));
        h2d(d, pending_init.data(), pending_init.size() * sizeof(ShardInit));
        hcheck(launch_shard_init(stream, (uint32_t)pending_init.size(), d));
        pending_init.clear();
        for (auto &ps : pending_state) h2d(ps.first, &ps.second, sizeof(ShardState));
        pending_state.clear();
    }

    // text-only arena of a PSA shard: the live chunk's docs (from hs.ctext_off: a rotation
    // inside a batch leaves the closed chunks' text in front of it) and room for B more bytes
    void text_reserve(Shard &s, uint64_t B) {
        const uint64_t live_off = s.text_only ? s.hs.ctext_off : 0;
        const uint64_t live = s.text_end - live_off;
        if (s.arena && s.text_only && live_off == 0 && s.text_end + B <= s.text_cap) return;
        const uint64_t need = live + B;
        const uint64_t cap = round_up(std::max(need, s.text_cap * 3 / 2) + 1024, 256);
        auto *a = (uint8_t *)heap.alloc(cap);
        if (s.arena) {
            if (live) hcheck(hipMemcpyAsync(a, s.text + live_off, live, hipMemcpyDeviceToDevice, stream));
            deferred_release.emplace_back(s.arena, s.arena_bytes);
        }
        s.text_end = live;
        s.hs.ctext_off = 0;
        s.arena = a;
        s.arena_bytes = cap;
        s.text = a;
        s.text_cap = cap - 1024;
        s.text_only = true;
        s.st = nullptr;
        s.root_tab = nullptr;
        s.doc_base = nullptr;
        s.nodes = nullptr;
        s.hash = nullptr;
        s.node_cap = s.doc_cap = 0;
        s.hash_cap = 0;
    }
    std::vector<std::pair<void *, uint64_t>> deferred_release;  // freed at the end of a set batch

    // a PSA shard's live chunk goes back to the walk: full arena, text copied, the live
    // docs' starts uploaded; returns the docs k_gst_encode must re-walk first
    uint32_t upgrade_to_walk(Shard &s, uint64_t B, uint32_t D) {
        std::vector<uint32_t> lens;
        if (s.hs.n_docs) {
            const Chunk &ch = chunks[s.chunks[s.hs.chunk_seq]];
            lens.assign(ch.doc_len.begin(), ch.doc_len.begin() + s.hs.n_docs);
        }
        return upgrade_to_walk(s, B, D, s.text_only ? s.hs.ctext_off : 0, lens);
    }
    // the live chunk's docs (lens) start at arena text offset live_off; everything from there
    // to text_end (this batch's docs included) moves to the walk's arena
    uint32_t upgrade_to_walk(Shard &s, uint64_t B, uint32_t D, uint64_t live_off, const std::vector<uint32_t> &lens) {
        const uint64_t live = s.text_end - live_off;
        const uint32_t docs = (uint32_t)lens.size();
        std::vector<uint32_t> base(docs + 1, 0);
        for (uint32_t i = 0; i < docs; ++i) base[i + 1] = base[i] + lens[i];
        void *old_arena = s.arena;
        const uint64_t old_bytes = s.arena_bytes;
        uint8_t *old_text = s.text;
        const uint32_t seq = s.hs.chunk_seq;
        s.arena = nullptr;
        s.text_only = false;
        s.psa = false;
        s.text_cap = 0;
        s.hs = ShardState{};
        s.hs.chunk_seq = seq;
        s.text_end = 0;
        shard_reserve(s, live + B, docs + D);
        if (live) hcheck(hipMemcpyAsync(s.text, old_text + live_off, live, hipMemcpyDeviceToDevice, stream));
        h2d(s.doc_base, base.data(), base.size() * 4);
        s.text_end = live;
        if (old_arena) deferred_release.emplace_back(old_arena, old_bytes);
        return docs;
    }

    // (re)build a shard's arena so the next batch (B new bytes, D new docs) fits
    void shard_reserve(Shard &s, uint64_t B, uint32_t D) {
        uint64_t need_nodes = std::min<uint64_t>((uint64_t)s.hs.n_nodes + 2 * B + 4, kChunkNodeCap);
        uint64_t need_docs = std::min<uint64_t>((uint64_t)s.hs.n_docs + D, kChunkSlots) + 1;
        uint64_t need_text = s.text_end + B;
        uint64_t need_hash = pow2_at_least(need_nodes);  // only 3rd+ children live in the hash
        bool fits = s.arena && need_nodes <= s.node_cap && need_docs <= s.doc_cap && need_text <= s.text_cap &&
                    need_hash <= s.hash_cap;
        if (fits) return;
        // new capacities (grow geometrically when the shard already exists)
        uint64_t g = s.arena ? 2 : 1;
        uint64_t node_cap = std::min<uint64_t>(std::max(need_nodes, (uint64_t)s.node_cap * g), kChunkNodeCap);
        uint64_t doc_cap = std::min<uint64_t>(std::max(need_docs, (uint64_t)s.doc_cap * g), kChunkSlots + 1);
        uint64_t live_text = s.text_end - s.hs.ctext_off;
        uint64_t text_cap = std::max(live_text + B, s.arena ? (live_text + B) * 3 / 2 : live_text + B);
        uint64_t hash_cap = pow2_at_least(node_cap);
        uint64_t off_root = round_up(sizeof(ShardState), 256);
        uint64_t off_doc = off_root + 256 * 16;
        uint64_t off_nodes = round_up(off_doc + (doc_cap + 1) * 4, 256);
        uint64_t off_hash = round_up(off_nodes + node_cap * 32, 256);
        uint64_t off_text = round_up(off_hash + hash_cap * 16, 256);
        uint64_t total = round_up(off_text + text_cap + 1024, 256);  // slack: the kernel's 256-byte doc window
        char *a = (char *)heap.alloc(total);
        Shard o = s;  // old view
        s.arena = a;
        s.arena_bytes = total;
        s.st = (ShardState *)a;
        s.root_tab = (uint4 *)(a + off_root);
        s.doc_base = (uint32_t *)(a + off_doc);
        s.nodes = (uint4 *)(a + off_nodes);
        s.hash = (uint4 *)(a + off_hash);
        s.text = (uint8_t *)(a + off_text);
        s.node_cap = (uint32_t)node_cap;
        s.doc_cap = (uint32_t)doc_cap - 1;
        s.hash_cap = hash_cap;
        s.text_cap = text_cap;
        if (!o.arena) {
            pending_init.push_back(ShardInit{s.hash, s.st, hash_cap});
            // a shard holding loaded chunks starts its GST in a fresh chunk after them
            if (s.hs.chunk_seq) pending_state.emplace_back(s.st, s.hs);
            s.text_end = 0;
            return;
        }
        hcheck(hipMemsetAsync(s.hash, 0, hash_cap * 16, stream));
        // migrate the live chunk: text moves to offset 0, everything else by copy / rehash
        hcheck(hipMemcpyAsync(s.root_tab, o.root_tab, 256 * 16, hipMemcpyDeviceToDevice, stream));
        hcheck(hipMemcpyAsync(s.doc_base, o.doc_base, ((size_t)o.hs.n_docs + 1) * 4, hipMemcpyDeviceToDevice, stream));
        hcheck(hipMemcpyAsync(s.nodes, o.nodes, (size_t)o.hs.n_nodes * 32, hipMemcpyDeviceToDevice, stream));
        hcheck(launch_rehash(stream, o.hash, (uint32_t)o.hash_cap, o.hs.epoch, s.hash, (uint32_t)(hash_cap - 1)));
        hcheck(hipMemcpyAsync(s.text, o.text + o.hs.ctext_off, live_text, hipMemcpyDeviceToDevice, stream));
        s.hs.ctext_off = 0;
        s.text_end = live_text;
        h2d(s.st, &s.hs, sizeof(ShardState));
        sync();
        heap.release(o.arena, o.arena_bytes);
    }

    // ------------------------------------------------------------ key prefixes
    const uint8_t *kp_of(const Leaf &l, uint32_t *len) const {
        const Chunk &c = chunks[l.chunk];
        *len = c.kp_len[l.idx];
        return reinterpret_cast<const uint8_t *>(c.kp.data()) + c.kp_off[l.idx];
    }

    // ------------------------------------------------------------ crit-bit ops
    // (the tree is px_host.h's CritBit; here: the stored key prefixes and what a replace /
    // delete does to the record)
    auto kp_fn() const {
        return [this](const Leaf &l, uint32_t *len) { return kp_of(l, len); };
    }
    // CritBitTree::setitem; q = escaped key incl. 251,0.  Returns 1 on replace.
    int cbt_insert(Shard &s, const std::string &q, Leaf nl) {
        const int rc = s.insert(q, nl, kp_fn(), [&](const Leaf &l) { chunk_delitem(s, l); });
        if (rc == 2) {  // (the shard's own chunks only: shards insert on separate host threads)
            Chunk &ch = chunks[nl.chunk];
            if (ch.notree.size() <= nl.idx) ch.notree.resize(nl.idx + 1, 0);
            ch.notree[nl.idx] = 1;
        } else if (!kp_matches(nl, q)) {
            s.unclean = true;
        }
        return rc;
    }

    // PiXiuChunk::delitem (PiXiuStr.cpp:178-187): dead mark, live count, Glob
    void chunk_delitem(Shard &s, const Leaf &l) {
        Chunk &ch = chunks[l.chunk];
        if (l.idx < ch.gid.size() && ch.gid[l.idx] != kNone) {  // (shards insert on several host threads)
            std::lock_guard<std::mutex> g(dki.mu);
            dki.kills.push_back(ch.gid[l.idx]);
        }
        if (!ch.dead[l.idx]) {
            ch.dead[l.idx] = 1;
            if (ch.used) ch.used--;
        }
        if (ch.used < 0.8 * kChunkSlots) s.glob = l.chunk;
    }

    // CritBitTree::getitem's key_eq (PiXiuStr.cpp:129-143) on the stored compat key prefix
    bool kp_matches(const Leaf &l, const std::string &q) const {
        uint32_t clen;
        const uint8_t *crit = kp_of(l, &clen);
        return pxh::CritBit::key_eq(crit, clen, q);
    }
    bool cbt_lookup(const Shard &s, const std::string &q, Leaf *out) const { return s.lookup(q, kp_fn(), out); }
    // CritBitTree::contains (CritBitTree.cpp:154-178): crit stream vs the escaped key bytes
    bool cbt_contains(const Shard &s, const std::string &q) const { return s.lookup(q, kp_fn(), nullptr); }
    // CritBitTree::delitem (CritBitTree.cpp:107-152)
    int cbt_delete(Shard &s, const std::string &q) {
        return s.remove(q, kp_fn(), [&](const Leaf &l) { chunk_delitem(s, l); });
    }

    // PiXiuStr::startswith (PiXiuStr.cpp:145-164) on a stored record: its stored compat
    // key prefix when that is long enough, else a GPU decode of the first |p| bytes
    bool rec_startswith(const Leaf &l, const std::string &p) {
        uint32_t klen;
        const uint8_t *kp = kp_of(l, &klen);
        if (p.size() <= klen) return memcmp(kp, p.data(), p.size()) == 0;
        std::vector<DecodeQuery> q{DecodeQuery{l.chunk, l.idx, 0, kMaxDoc, 0, (uint32_t)p.size(), 0}};
        auto *d = (uint8_t *)iter_buf.get(round_up(p.size(), 64) + 64);
        std::vector<uint32_t> len, st;
        run_decode(q, d, len, st, false);
        if ((st[0] != kOk && st[0] != kErrSpace) || len[0] < p.size()) return false;
        std::string got(p.size(), '\0');
        d2h(&got[0], d, p.size());
        sync();
        return got == p;
    }

    // CritBitTree::iter (CBTGHelper / CBTGen, CritBitTree.h:55-157); the first leaf
    // reached must start with the prefix (rec_startswith)
    bool cbt_iter(const Shard &s, const std::string &p, std::vector<Leaf> &out) {
        return s.iter(p, [&](const Leaf &l) { return rec_startswith(l, p); }, out);
    }

    // the escaped key the CritBit stores (raw bytes, 251 doubled, then 251,0), built
    // into q (reused buffers keep lookups off the allocator)
    static void esc_key_into(std::string &q, const uint8_t *k, uint64_t n) {
        q.clear();
        const uint8_t *e = (const uint8_t *)std::memchr(k, kEsc, n);
        if (!e) {
            q.append(reinterpret_cast<const char *>(k), n);
        } else {
            q.reserve(n + 8);
            for (uint64_t i = 0; i < n; ++i) {
                q.push_back((char)k[i]);
                if (k[i] == kEsc) q.push_back((char)kEsc);
            }
        }
        q.push_back((char)kEsc);
        q.push_back((char)kKeyEnd);
    }
    static std::string esc_key(const uint8_t *k, uint64_t n) {
        std::string q;
        esc_key_into(q, k, n);
        return q;
    }
    // the CritBit key of a set input: the escaped key, or a ready doc's prefix through its
    // first 251,0 (raw_docs)
    std::string crit_key(const uint8_t *k, uint64_t n) const;

    Shard *shard_for_key(const uint8_t *k, uint64_t n) const {
        if (opts.records_per_shard == 0) return shards.empty() ? nullptr : shards[0].get();
        const int64_t s = keymap.find(k, n);
        return s < 0 ? nullptr : shards[(size_t)s].get();
    }

    // ------------------------------------------------------------ decode
    // Runs decode queries; out_dev is a device buffer.  Returns per-query len/status.
    static bool spans_enabled() {  // PX_SPANS=0: no span tables, every getitem walks
        const char *e = std::getenv("PX_SPANS");
        return !(e && e[0] == '0');
    }
    // the table serving query q: {entries, count, expansion length}, or entries == null
    struct SpanView {
        const SpanEnt *p;
        const uint32_t *t;
        uint32_t n, len;
    };
    SpanView span_view(const DecodeQuery &q) const {
        if (q.chunk == kNone || q.from != 0 || q.to < kMaxDoc) return SpanView{nullptr, nullptr, 0, 0};
        const Chunk &ch = chunks[q.chunk];
        if (q.idx >= ch.span.size()) return SpanView{nullptr, nullptr, 0, 0};
        const Chunk::Span &sp = ch.span[q.idx];
        if (!sp.p) return SpanView{nullptr, nullptr, 0, 0};
        if (q.mode == 0 || sp.eq) return SpanView{sp.p, sp.t, sp.n, sp.len};
        return SpanView{sp.xp, sp.xt, sp.xn, sp.xlen};
    }

    // Full-range getitem queries on records with span tables go to k_gather: they are
    // taken out of qn[lo, hi) (chunk -> kNone: k_decode's wave skips them) and returned
    // as gather queries whose result slot is their position in the launch's arrays.
    std::vector<GatherQuery> take_gathers(DecodeQuery *qn, uint32_t lo, uint32_t hi, uint32_t slot0) {
        std::vector<GatherQuery> g;
        if (!spans_enabled()) return g;
        for (uint32_t j = lo; j < hi; ++j) {
            const SpanView sp = span_view(qn[j]);
            if (!sp.p) continue;
            g.push_back(GatherQuery{sp.p, chunks[qn[j].chunk].slots[qn[j].idx].comp, qn[j].out_off, sp.n, sp.len,
                                    qn[j].out_cap, j - lo + slot0, sp.t, 0, 0});
            qn[j].chunk = kNone;
            qn[j].nrec = 0;
        }
        return g;
    }
    // take_gathers with the queries prepared by the resolving threads (pg: span == nullptr
    // where the record has no table)
    std::vector<GatherQuery> take_gathers_pre(DecodeQuery *qn, uint32_t lo, uint32_t hi, const GatherQuery *pg) {
        std::vector<GatherQuery> g;
        g.reserve(hi - lo);
        for (uint32_t j = lo; j < hi; ++j) {
            if (!pg[j].span || qn[j].chunk == kNone) continue;
            g.push_back(pg[j]);
            g.back().out_off = qn[j].out_off;
            g.back().slot = j - lo;
            qn[j].chunk = kNone;
            qn[j].nrec = 0;
        }
        return g;
    }
    // after the k_decode launch on the same stream (its skipped-query results are overwritten).
    // The launch's tiles (a tile = kGatherTile output bytes of one query; a query's tiles
    // are consecutive) go 64 to a wave, across queries when they are small; the queries go
    // up from pinned memory (`which`: the launch's own staging buffer) and k_gather_tasks
    // finds each wave's first query on the device.
    void launch_gathers(hipStream_t st, std::vector<GatherQuery> &g, uint8_t *out, uint32_t *dl, uint32_t *ds,
                        GatherQuery *&dbuf, int which) {
        if (g.empty()) return;
        uint32_t tiles = 0;
        for (auto &q : g) {
            q.tile0 = tiles;
            tiles += std::max<uint32_t>(1, (std::min(q.len, q.cap) + kGatherTile - 1) / kGatherTile);  // (>= 1: the status)
        }
        const uint32_t ntask = (tiles + 63) / 64;
        const uint64_t qb = round_up(g.size() * sizeof(GatherQuery), 64);
        auto *hg = (GatherQuery *)hg_buf[which].get(g.size() * sizeof(GatherQuery));
        std::memcpy(hg, g.data(), g.size() * sizeof(GatherQuery));
        dbuf = (GatherQuery *)heap.alloc(qb + gather_task_bytes(ntask));
        void *task = (uint8_t *)dbuf + qb;  // per task: GatherTask
        hcheck(hipMemcpyAsync(dbuf, hg, g.size() * sizeof(GatherQuery), hipMemcpyHostToDevice, st));
        hcheck(launch_gather(st, ntask, nullptr, 0, task, dbuf, (uint32_t)g.size(), out, dl, ds));
        gather_bytes[dbuf] = qb + gather_task_bytes(ntask);
    }
    std::map<void *, uint64_t> gather_bytes;  // launch_gathers' device buffers -> their sizes
    void release_gathers(GatherQuery *d) {
        if (!d) return;
        auto it = gather_bytes.find(d);
        heap.release(d, it->second);
        gather_bytes.erase(it);
    }

    // Runs decode queries; out_dev is a device buffer.  Returns per-query len/status.
    // getitem batches (timed) send span-served queries to k_gather.
    void run_decode(const std::vector<DecodeQuery> &q, uint8_t *out_dev, std::vector<uint32_t> &len,
                    std::vector<uint32_t> &st, bool timed) {
        uint32_t nq = (uint32_t)q.size();
        len.assign(nq, 0);
        st.assign(nq, 0);
        if (!nq) return;
        uint32_t depth = opts.decode_depth ? opts.decode_depth : 4096;
        // auto: one wave per query up to 16,384 (measured on config 3: 10k queries take
        // 6.27 ms on 8,192 waves, 5.96 ms on one wave each)
        uint32_t waves = opts.decode_waves ? opts.decode_waves : 16384;
        waves = std::min(waves, nq);
        auto *frames = (Frame *)scratch_frames.get((uint64_t)waves * depth * sizeof(Frame));
        auto *dq = (DecodeQuery *)dq_buf.get((uint64_t)nq * sizeof(DecodeQuery));
        auto *dl = (uint32_t *)dlen_buf.get((uint64_t)nq * 8);
        uint32_t *ds = dl + nq;
        auto *qn = (DecodeQuery *)hq_buf.get((uint64_t)nq * sizeof(DecodeQuery));
        // queries grouped by chunk (stable), so that one chunk's queries run together on
        // one XCD (k_decode's remap); results are mapped back below
        std::vector<uint32_t> perm;
        bool sorted = true;
        for (uint32_t i = 1; i < nq && sorted; ++i) sorted = q[i - 1].chunk <= q[i].chunk;
        if (!sorted) {
            perm.resize(nq);
            for (uint32_t i = 0; i < nq; ++i) perm[i] = i;
            std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) { return q[a].chunk < q[b].chunk; });
        }
        parallel_ranges(nq, nq >= 65536 ? host_threads() : 1, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t j = lo; j < hi; ++j) {
                const DecodeQuery &src = q[perm.empty() ? j : perm[j]];
                qn[j] = src;
                qn[j].nrec = src.chunk == kNone ? 0 : chunks[src.chunk].n;
            }
        });
        std::vector<GatherQuery> gq;
        if (timed) gq = take_gathers(qn, 0, nq, 0);
        stats.last_gather_queries = timed ? (uint32_t)gq.size() : stats.last_gather_queries;
        // every found key gathered: no walk launch (the host answers the missing keys)
        bool walk = false;
        for (uint32_t j = 0; j < nq && !walk; ++j) walk = qn[j].chunk != kNone;
        if (walk) hcheck(hipMemcpyAsync(dq, qn, (size_t)nq * sizeof(DecodeQuery), hipMemcpyHostToDevice, stream));
        flush_tab();
        if (timed) hcheck(hipEventRecord(ev0, stream));
        // timed == a getitem batch (k_decode); otherwise stored-key prefixes (k_decode_keys)
        static const bool xcd = [] {
            const char *e = std::getenv("PX_DEC_XCD");
            return !(e && e[0] == '0');
        }();
        if (!walk) {
        } else {
            hcheck(launch_decode(stream, dq, nq, (const RecSlot *const *)chunk_tab, out_dev, dl, ds, frames, depth,
                                 waves | (xcd ? 0x80000000u : 0u), !timed));
        }
        GatherQuery *dgq = nullptr;
        launch_gathers(stream, gq, out_dev, dl, ds, dgq, 0);
        if (timed) hcheck(hipEventRecord(ev1, stream));
        auto *hr = (uint32_t *)hres_buf.get((uint64_t)nq * 8);
        hcheck(hipMemcpyAsync(hr, dl, (size_t)nq * 8, hipMemcpyDeviceToHost, stream));  // lengths, then statuses
        sync();
        release_gathers(dgq);
        if (timed) {
            float ms = 0;
            hcheck(hipEventElapsedTime(&ms, ev0, ev1));
            stats.last_decode_kernel_ms = ms;
        }
        if (perm.empty()) {
            std::memcpy(len.data(), hr, (size_t)nq * 4);
            std::memcpy(st.data(), hr + nq, (size_t)nq * 4);
        } else {
            for (uint32_t j = 0; j < nq; ++j) {
                len[perm[j]] = hr[j];
                st[perm[j]] = hr[nq + j];
            }
        }
    }

    // Span tables for new records: k_decode_addr -> k_span_jobs count -> two scans -> (one
    // round trip: counts and lengths down, the table allocated) -> k_span_jobs write.  The
    // jobs are built on the device from the decode's own queries, in chunk order.  docs: each
    // record's escaped doc on the device (for the compat == exact flag), or null.  A record
    // whose compat expansion overran its doc + 64 bytes, or reaches a source beyond +-2 GiB,
    // keeps using the walk.
    struct SpanReq {
        uint32_t chunk, idx;
        const uint8_t *doc;
    };
    void build_spans(const std::vector<SpanReq> &reqs_in, uint32_t mode = 0, bool exact_too = true, bool split = true) {
        if (reqs_in.empty() || !spans_enabled()) return;
        std::vector<SpanReq> sorted_reqs;
        const std::vector<SpanReq> *rp = &reqs_in;
        for (size_t k = 1; k < reqs_in.size(); ++k)
            if (reqs_in[k].chunk < reqs_in[k - 1].chunk) {  // (k_decode's XCD grouping wants chunk order)
                sorted_reqs = reqs_in;
                std::stable_sort(sorted_reqs.begin(), sorted_reqs.end(),
                                 [](const SpanReq &x, const SpanReq &y) { return x.chunk < y.chunk; });
                rp = &sorted_reqs;
                break;
            }
        const std::vector<SpanReq> &reqs = *rp;
        const uint32_t n = (uint32_t)reqs.size();
        PhaseClock phase(mode ? "build_spans (exact)" : "build_spans", "PX_SET_VERBOSE");
        phase.mark("queries and sources");
        // queries (pinned) and sources
        // Records are decoded in pieces of kPiece source bytes, one wave each (a config-3 batch
        // has 10,000 records of 60 KB: whole, their waves kept the decode at 19 ms).
        //  * exact: an exact parse of [a, b) of a record whose exact expansion is its doc is the
        //    doc's slice, so the pieces' addresses land side by side; a record whose pieces do
        //    not reassemble its doc (one near a length-251 alias token: its exact expansion is
        //    not its doc, and its doc coordinates are not the decoder's) is decoded again whole;
        //  * compat: pieces are cut at token starts (k_span_pieces) and carry the whole drain's
        //    ret cursor, so each drains the same top-level tokens as the whole drain, to the
        //    same bytes; each lands 64 bytes past the previous piece's nominal end (an
        //    over-yield has room) and k_span_jobs reads the pieces in order.  A record whose
        //    pieces fail or reach the whole decode's room is decoded again whole.
        static const uint32_t kPiece = [] {  // (PX_SPAN_PIECE: experiments; a power of two >= 256)
            const char *e = std::getenv("PX_SPAN_PIECE");
            const uint32_t v = e ? (uint32_t)std::atoi(e) : 4096u;
            return v >= 256 && (v & (v - 1)) == 0 ? v : 4096u;
        }();
        const char *split_env = std::getenv("PX_SPAN_SPLIT");
        const bool compat_split = !(split_env && split_env[0] == '0');
        split = split && (mode == 1 || compat_split);
        // sources in pinned memory (copied to the device from there), filled on host threads with
        // every record's doc length; the offsets by a parallel prefix (a million-record batch spent
        // ~3.7 ms here in serial loops and a staged copy)
        const uint32_t pthr = n >= 65536 ? host_threads() : 1;
        auto *src = static_cast<SpanSrc *>(src_pin.get((uint64_t)n * sizeof(SpanSrc) + 64));
        std::atomic<bool> longer{false};
        parallel_ranges(n, pthr, [&](uint32_t lo, uint32_t hi) {
            bool lg = false;
            for (uint32_t k = lo; k < hi; ++k) {
                const uint32_t L = chunks[reqs[k].chunk].doc_len[reqs[k].idx];
                src[k] = SpanSrc{reqs[k].doc, L, 0};
                lg = lg || L > kPiece;
            }
            if (lg) longer.store(true);
        });
        split = split && longer.load();  // (a batch whose records are all one piece long: whole decodes, no piece table)
        auto *qn = (DecodeQuery *)hq_buf.get((uint64_t)n * sizeof(DecodeQuery));
        std::vector<uint64_t> qoff(n + 1);
        pxh::parallel_prefix(n, pthr, qoff.data(), [&](uint32_t k) -> uint64_t {
            const uint32_t L = src[k].doc_len;
            return round_up(L + 64, 16) + (split && mode == 0 ? 64ull * std::max<uint32_t>(1, (L + kPiece - 1) / kPiece) : 0ull);
        });
        const uint64_t tot = qoff[n];
        parallel_ranges(n, pthr, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t k = lo; k < hi; ++k) {
                const SpanReq &r = reqs[k];
                const Chunk &ch = chunks[r.chunk];
                const uint32_t cap = (uint32_t)round_up(src[k].doc_len + 64, 16);
                qn[k] = DecodeQuery{r.chunk, r.idx, 0, kMaxDoc, qoff[k], cap, mode, ch.n, 0};
            }
        });
        auto *addr = (int32_t *)heap.alloc(tot * 4 + 64);
        hcheck(hipMemsetD32Async((hipDeviceptr_t)addr, kAddrMark, tot, stream));  // (k_decode_addr writes run starts only)
        // device: queries, lengths + statuses, sources, counts / entries / tiles and their scans
        const uint64_t o_dl = round_up((uint64_t)n * sizeof(DecodeQuery), 256), o_src = o_dl + round_up((uint64_t)n * 8, 256),
                       o_u32 = o_src + round_up((uint64_t)n * sizeof(SpanSrc), 256), o_end = o_u32 + (uint64_t)n * 20 + 256;
        auto *wb = (uint8_t *)heap.alloc(o_end);
        auto *dq = (DecodeQuery *)wb;
        auto *dl = (uint32_t *)(wb + o_dl), *ds = dl + n;
        auto *dsrc = (SpanSrc *)(wb + o_src);
        auto *cnt = (uint32_t *)(wb + o_u32), *ents = cnt + n, *tiles = ents + n, *eoff = tiles + n, *toff = eoff + n;
        phase.mark("uploads, decode, count, scans");
        hcheck(hipMemcpyAsync(dq, qn, (size_t)n * sizeof(DecodeQuery), hipMemcpyHostToDevice, stream));
        hcheck(hipMemcpyAsync(dsrc, src, (size_t)n * sizeof(SpanSrc), hipMemcpyHostToDevice, stream));
        flush_tab();
        const uint32_t depth = opts.decode_depth ? opts.decode_depth : 4096;
        const uint32_t waves = std::min<uint32_t>(opts.decode_waves ? opts.decode_waves : 16384, n);
        auto *frames = (Frame *)scratch_frames.get((uint64_t)waves * depth * sizeof(Frame));
        static const bool xcd = [] {
            const char *e = std::getenv("PX_DEC_XCD");
            return !(e && e[0] == '0');
        }();
        const auto *ctab = (const RecSlot *const *)chunk_tab;
        uint64_t sub_bytes = 0;
        uint8_t *sub_buf = nullptr;
        DecodeQuery *sdq = nullptr;
        uint32_t *dfirst = nullptr, *pl = nullptr;
        if (split) {
            // every record's pieces: counts, their prefix, then the queries written straight into
            // pinned memory on host threads (a staged copy of the piece table left the GPU idle
            // ~2 ms on config 3)
            std::vector<uint32_t> first(n + 1, 0);
            for (uint32_t k = 0; k < n; ++k) {
                const uint32_t L = src[k].doc_len;
                first[k + 1] = first[k] + (L == 0 ? 1u : (L + kPiece - 1) / kPiece);
            }
            auto *sq = static_cast<DecodeQuery *>(piece_pin.get((uint64_t)first[n] * sizeof(DecodeQuery) + 64));
            parallel_ranges(n, pthr, [&](uint32_t lo, uint32_t hi) {
                for (uint32_t k = lo; k < hi; ++k) {
                    const uint32_t L = src[k].doc_len;
                    DecodeQuery *o = sq + first[k];
                    for (uint32_t a = 0, m = 0; a < L || (a == 0 && L == 0); a += kPiece, ++m) {
                        const uint32_t b = std::min(L, a + kPiece);
                        DecodeQuery d = qn[k];
                        d.from = (int32_t)a;
                        d.to = (int32_t)b;
                        if (mode == 1) {
                            d.out_off = qn[k].out_off + a;
                            d.out_cap = b - a + 16;  // (exactly b - a bytes come; room past them keeps the cap from firing)
                        } else {
                            d.out_off = qn[k].out_off + 64ull * m;  // (k_span_pieces adds the piece's start)
                            d.pad = L;
                        }
                        o[m] = d;
                        if (L == 0) break;
                    }
                }
            });
            const uint32_t ns = first[n];
            const uint64_t o_first = round_up((uint64_t)ns * sizeof(DecodeQuery), 256);
            const uint64_t o_pl = o_first + round_up((uint64_t)(n + 1) * 4, 256);
            sub_bytes = o_pl + (uint64_t)ns * 8 + 256;
            sub_buf = (uint8_t *)heap.alloc(sub_bytes);
            sdq = (DecodeQuery *)sub_buf;
            dfirst = (uint32_t *)(sub_buf + o_first);
            pl = (uint32_t *)(sub_buf + o_pl);
            uint32_t *ps = pl + ns;
            hcheck(hipMemcpyAsync(sdq, sq, (size_t)ns * sizeof(DecodeQuery), hipMemcpyHostToDevice, stream));
            h2d(dfirst, first.data(), (size_t)(n + 1) * 4);
            if (mode == 0) hcheck(launch_span_pieces(stream, ns, sdq, ctab, kPiece));
            const uint32_t sw = std::min<uint32_t>(opts.decode_waves ? opts.decode_waves : 16384, ns);
            auto *sframes = (Frame *)scratch_frames.get((uint64_t)sw * depth * sizeof(Frame));
            // (the pieces in launch order: the XCD remap measured 0.65 ms slower here -- config 3's
            // decode + count 13.6 against 12.9 ms over 6 and 4 batches, CHANGELOG round 6; the
            // pieces' tail, not L2 locality, bounds this decode.  PX_SPAN_XCD=1 restores it)
            static const bool span_xcd = [] {
                const char *e = std::getenv("PX_SPAN_XCD");
                return e && e[0] == '1';
            }();
            hcheck(launch_decode_addr(stream, sdq, ns, ctab, addr, pl, ps, sframes, depth, sw | (span_xcd ? 0x80000000u : 0u)));
            hcheck(launch_span_agg(stream, n, dfirst, pl, ps, dq, dl, ds));
        } else {
            hcheck(launch_decode_addr(stream, dq, n, ctab, addr, dl, ds, frames, depth, waves | (xcd ? 0x80000000u : 0u)));
        }
        hcheck(launch_span_jobs(stream, n, dq, dl, ds, dsrc, ctab, addr, cnt, ents, tiles, nullptr, nullptr, nullptr,
                                nullptr, sdq, pl, dfirst));
        const SortAlloc SA{[](void *self, uint64_t bytes) -> void * { return static_cast<px_ctx *>(self)->heap.alloc(bytes); },
                           [](void *self, void *p, uint64_t bytes) { static_cast<px_ctx *>(self)->heap.release(p, bytes); },
                           this};
        hcheck(scan_u32(stream, SA, ents, eoff, n, ScanOp::kPlus, false));
        hcheck(scan_u32(stream, SA, tiles, toff, n, ScanOp::kPlus, false));
        // counts and lengths down (one round trip)
        auto *hr = (uint32_t *)hres_buf.get((uint64_t)n * 8 + 16);
        hcheck(hipMemcpyAsync(hr, cnt, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
        hcheck(hipMemcpyAsync(hr + n, dl, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
        phase.mark("wait (decode + count)");
        hcheck(hipStreamSynchronize(stream));
        phase.mark("table sizes, write pass, views");
        const uint32_t *hc = hr, *hl = hr + n;
        if (std::getenv("PX_SPAN_VERBOSE")) {  // (diagnostics: why records get no table)
            std::vector<uint32_t> hs(n);
            hcheck(hipMemcpy(hs.data(), ds, (size_t)n * 4, hipMemcpyDeviceToHost));
            std::map<uint32_t, uint32_t> why;
            uint32_t bad = 0;
            for (uint32_t j = 0; j < n; ++j)
                if (hc[j] & kSpanBad) {
                    ++bad;
                    ++why[hs[j]];
                    if (bad <= 5)
                        fprintf(stderr, "span: no table for chunk %u idx %u: decode status %u len %u doc_len %u\n",
                                reqs[j].chunk, reqs[j].idx, hs[j], hl[j], chunks[reqs[j].chunk].doc_len[reqs[j].idx]);
                }
            fprintf(stderr, "span: mode %u, %u records, %u without a table:", mode, n, bad);
            for (auto &w : why) fprintf(stderr, " status %u x%u", w.first, w.second);
            fprintf(stderr, "\n");
        }
        // split decodes to do again whole: exact ones that are not the doc, compat ones that
        // failed (the whole decode decides those records)
        std::vector<SpanReq> redo;
        std::vector<uint8_t> skip(n, 0);
        if (split)
            for (uint32_t j = 0; j < n; ++j) {
                const bool bad = (hc[j] & kSpanBad) != 0;
                if (mode == 0 ? bad : (!bad && (!(hc[j] & kSpanEq) || hl[j] != src[j].doc_len))) {
                    redo.push_back(reqs[j]);
                    skip[j] = 1;
                }
            }
        std::vector<uint8_t> need_x(n, 0);  // compat tables that are not the doc: an exact table too
        uint64_t nents = 0, ntiles = 0;
        {
            std::vector<uint64_t> part_e(pthr > 1 ? 64 : 1, 0), part_t(part_e.size(), 0);
            const uint32_t np = (uint32_t)part_e.size(), per = (n + np - 1) / np;
            const std::function<void(uint32_t)> cnt_job = [&](uint32_t t) {
                uint64_t ce = 0, ct = 0;
                for (uint32_t j = t * per, e = std::min(n, j + per); j < e; ++j)
                    if (!(hc[j] & kSpanBad)) {
                        ce += (hc[j] & ~(kSpanBad | kSpanEq)) + 1;
                        ct += (hl[j] + kGatherTile - 1) / kGatherTile;
                    }
                part_e[t] = ce;
                part_t[t] = ct;
            };
            if (np > 1) WorkerPool::get().run(np, cnt_job);
            else cnt_job(0);
            for (uint32_t t = 0; t < np; ++t) nents += part_e[t], ntiles += part_t[t];
        }
        if (nents) {
            // entries, then every record's tile index (4 B per kGatherTile output bytes); the
            // host's running offsets are the device scans' (same counts, same order)
            const uint64_t tab_bytes = round_up(nents * sizeof(SpanEnt), 64) + ntiles * 4 + 64;
            auto *tab = (SpanEnt *)heap.alloc(tab_bytes);
            store_blocks.emplace_back(tab, tab_bytes);
            macct.span += tab_bytes;
            auto *tixb = (uint32_t *)((uint8_t *)tab + round_up(nents * sizeof(SpanEnt), 64));
            hcheck(launch_span_jobs(stream, n, dq, dl, ds, dsrc, ctab, addr, cnt, ents, tiles, eoff, toff, tab, tixb, sdq,
                                    pl, dfirst));
            // every record's entry and tile offsets (the device scans' running sums), the
            // chunks' view tables sized, then the views filled on host threads
            std::vector<uint64_t> eo(n + 1), tofs(n + 1);
            pxh::parallel_prefix(n, pthr, eo.data(), [&](uint32_t j) -> uint64_t {
                return (hc[j] & kSpanBad) ? 0u : (hc[j] & ~(kSpanBad | kSpanEq)) + 1u;
            });
            pxh::parallel_prefix(n, pthr, tofs.data(), [&](uint32_t j) -> uint64_t {
                return (hc[j] & kSpanBad) ? 0u : (hl[j] + kGatherTile - 1) / kGatherTile;
            });
            uint64_t used = eo[n];
            for (uint32_t j = 0; j < n; ++j)
                if (skip[j]) used -= eo[j + 1] - eo[j];
            {
                // (the requests come in chunk order: one check per chunk; the chunks' view tables
                // sized on host threads -- value-initialising a new chunk's table is page faults)
                std::vector<uint32_t> cs;
                for (uint32_t j = 0; j < n; ++j)
                    if (j == 0 || reqs[j].chunk != reqs[j - 1].chunk) cs.push_back(reqs[j].chunk);
                const std::function<void(uint32_t)> rs = [&](uint32_t i) {
                    Chunk &ch = chunks[cs[i]];
                    if (ch.span.size() < ch.n) ch.span.resize(ch.n);
                };
                if (cs.size() > 4 && n >= 65536) WorkerPool::get().run((uint32_t)cs.size(), rs);
                else for (uint32_t i = 0; i < (uint32_t)cs.size(); ++i) rs(i);
            }
            stats.span_entries += used;
            parallel_ranges(n, pthr, [&](uint32_t lo, uint32_t hi) {
                for (uint32_t j = lo; j < hi; ++j) {
                    // (a skipped record's entries are written but not used: the whole decode
                    // replaces them)
                    if ((hc[j] & kSpanBad) || skip[j]) continue;
                    Chunk &ch = chunks[reqs[j].chunk];
                    const uint32_t ns = hc[j] & ~(kSpanBad | kSpanEq);
                    Chunk::Span &sp = ch.span[reqs[j].idx];
                    if (mode == 0) {
                        sp.p = tab + eo[j];
                        sp.t = tixb + tofs[j];
                        sp.n = ns;
                        sp.len = hl[j];
                        sp.eq = (hc[j] & kSpanEq) != 0;
                        if (!sp.eq) need_x[j] = 1;
                    } else {
                        sp.xp = tab + eo[j];
                        sp.xt = tixb + tofs[j];
                        sp.xn = ns;
                        sp.xlen = hl[j];
                    }
                }
            });
        }
        phase.mark("wait (write pass)");
        sync();
        if (sub_buf) heap.release(sub_buf, sub_bytes);
        heap.release(wb, o_end);
        heap.release(addr, tot * 4 + 64);
        if (!redo.empty()) build_spans(redo, mode, false, false);
        phase.mark("exact tables");
        if (mode == 0 && exact_too) {  // exact tables for the records whose compat expansion is not the doc
            // (marked while the views were filled; a record the whole decode redid is checked here)
            std::vector<SpanReq> x;
            for (uint32_t j = 0; j < n; ++j) {
                if (!need_x[j] && !skip[j]) continue;
                const SpanReq &r = reqs[j];
                const Chunk &ch = chunks[r.chunk];
                if (r.idx < ch.span.size() && ch.span[r.idx].p && !ch.span[r.idx].eq) x.push_back(r);
            }
            build_spans(x, 1);
        }
    }

    // key -> decode query (CritBit lookup, CritBitTree.cpp:13-40); pre = PX_ENOTFOUND when absent
    void resolve_key(const uint8_t *k, uint64_t kn, int mode, std::string &ek, DecodeQuery &q, uint32_t &pre) const {
        esc_key_into(ek, k, kn);
        q = DecodeQuery{kNone, 0, 0, kMaxDoc, 0, 0, (uint32_t)mode};
        pre = PX_OK;
        const Shard *s = nullptr;
        if (opts.records_per_shard != 0) {
            // the key map's record hint: a live record whose stored key equals the query
            // is the one the CritBit walk would reach (a trie holds one live leaf per key)
            uint32_t sh, c, i;
            if (!keymap.find_hint(k, kn, &sh, &c, &i)) {
                pre = PX_ENOTFOUND;
                return;
            }
            // (only while that record is in its shard's trie and the trie holds clean prefixes
            // only: the reference skips some inserts, CritBitTree.cpp:96-100)
            if (c < chunks.size() && i < chunks[c].n && !chunks[c].dead[i] && chunks[c].in_tree(i) &&
                !shards[sh]->unclean && kp_matches(Leaf{c, i}, ek)) {
                q.chunk = c;
                q.idx = i;
                q.out_cap = (uint32_t)round_up(chunks[c].doc_len[i] + 64, 16);
                return;
            }
            s = shards[sh].get();
        } else {
            s = shard_for_key(k, kn);
        }
        Leaf l;
        if (!s || !cbt_lookup(*s, ek, &l)) {
            pre = PX_ENOTFOUND;
            return;
        }
        q.chunk = l.chunk;
        q.idx = l.idx;
        q.out_cap = (uint32_t)round_up(chunks[l.chunk].doc_len[l.idx] + 64, 16);
    }

    // resolve_key over keys [lo, hi) with the key map's cache misses overlapped: the hashes
    // of the next kAhead keys are computed and their first probe slots prefetched, then the
    // hinted record's chunk metadata and key prefix, so each key's lookup finds its lines in
    // cache (a lone lookup is a chain of ~6 dependent misses)
    void resolve_range(uint32_t lo, uint32_t hi, const uint8_t *keys, const uint64_t *koff, int mode,
                       DecodeQuery *q, uint32_t *pre) {
        std::string ek;
        if (opts.records_per_shard == 0 || hi - lo < 64) {
            for (uint32_t i = lo; i < hi; ++i) resolve_key(keys + koff[i], koff[i + 1] - koff[i], mode, ek, q[i], pre[i]);
            return;
        }
        constexpr uint32_t kAhead = 16;
        uint64_t hs[2 * kAhead];
        auto stage1 = [&](uint32_t i) {  // hash, prefetch the probe slot
            const uint64_t h = pxh::KeyMap::hash(keys + koff[i], koff[i + 1] - koff[i]);
            hs[i % (2 * kAhead)] = h;
            if (const void *a = keymap.slot_addr(h)) __builtin_prefetch(a);
        };
        auto stage2 = [&](uint32_t i) {  // the hinted record's metadata and key prefix
            uint32_t sh, c, x;
            if (keymap.find_hint_h(hs[i % (2 * kAhead)], keys + koff[i], koff[i + 1] - koff[i], &sh, &c, &x) &&
                c < chunks.size() && x < chunks[c].n) {
                const Chunk &ch = chunks[c];
                __builtin_prefetch(&ch.dead[x]);
                __builtin_prefetch(&ch.doc_len[x]);
                __builtin_prefetch(&ch.kp_off[x]);
                __builtin_prefetch(&ch.kp_len[x]);
            }
        };
        const uint32_t pro = std::min(hi, lo + kAhead);
        for (uint32_t i = lo; i < pro; ++i) stage1(i);
        for (uint32_t i = lo; i < hi; ++i) {
            if (i + kAhead < hi) stage1(i + kAhead);
            if (i + kAhead / 2 < hi) stage2(i + kAhead / 2);
            resolve_key(keys + koff[i], koff[i + 1] - koff[i], mode, ek, q[i], pre[i]);
        }
    }

    // share of a get batch (in 64ths) resolved before the first decode launch
    static uint32_t opts_head_frac() {
        static const uint32_t f = [] {
            const char *e = std::getenv("PX_GET_HEAD64");
            const int v = e ? std::atoi(e) : 0;
            return v > 0 && v < 64 ? (uint32_t)v : 24u;
        }();
        return f;
    }

    // getitem into a device buffer with the host key lookups overlapped with k_decode:
    // the first `head` keys are resolved and their decode launched at once; the rest
    // are resolved on host threads while the GPU expands the head, then launched on a
    // second stream, so the two launches share the GPU (the head alone does not fill
    // it).  Same results as resolving everything first and calling expand().
    int get_overlapped(uint32_t n, const uint8_t *keys, const uint64_t *koff, int mode, uint8_t *out,
                       uint64_t out_cap, uint64_t *out_off, uint32_t *out_len, uint32_t *status, uint64_t *needed,
                       double &lookup_ms) {
        using clk = std::chrono::steady_clock;
        std::vector<DecodeQuery> q(n);
        std::vector<uint32_t> pre(n, PX_OK);
        // each key's gather query too (span table, compressed base), on the same host threads:
        // its chunk metadata is in the resolving thread's cache, and the serial
        // take_gathers_pre below then only reads this array
        std::unique_ptr<GatherQuery[]> pg(new GatherQuery[n]);
        const bool spans = spans_enabled();
        auto resolve = [&](uint32_t lo, uint32_t hi) {
            resolve_range(lo, hi, keys, koff, mode, q.data(), pre.data());
            for (uint32_t j = lo; j < hi; ++j) {
                pg[j].span = nullptr;
                if (!spans || q[j].chunk == kNone) continue;
                const SpanView sp = span_view(q[j]);
                if (!sp.p) continue;
                pg[j] = GatherQuery{sp.p, chunks[q[j].chunk].slots[q[j].idx].comp, 0, sp.n, sp.len, q[j].out_cap, 0,
                                    sp.t, 0, 0};
            }
        };
        uint64_t total = 0;
        auto place = [&](uint32_t lo, uint32_t hi) {  // output offsets, in key order
            for (uint32_t i = lo; i < hi; ++i) {
                out_off[i] = total;
                q[i].out_off = total;
                q[i].nrec = q[i].chunk == kNone ? 0 : chunks[q[i].chunk].n;
                if (q[i].chunk != kNone) total += q[i].out_cap;
            }
        };
        const uint32_t head = std::max<uint32_t>(1024, (uint32_t)((uint64_t)n * opts_head_frac() / 64));
        PhaseClock phase("get_overlapped", "PX_GET_VERBOSE");
        phase.mark("head lookups");
        auto t0 = clk::now();
        parallel_ranges(head, host_threads(), [&](uint32_t lo, uint32_t hi) { resolve(lo, hi); });
        place(0, head);
        double head_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        if (total > out_cap) {  // cannot launch the head: plain path (reports PX_ESPACE)
            parallel_ranges(n - head, host_threads(), [&](uint32_t lo, uint32_t hi) { resolve(head + lo, head + hi); });
            lookup_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
            return expand(q, out, out_cap, 1, out_off, out_len, status, needed, pre);
        }
        const uint32_t depth = opts.decode_depth ? opts.decode_depth : 4096;
        const uint32_t w1 = std::min<uint32_t>(16384, head), w2 = std::min<uint32_t>(16384, n - head);
        auto *frames = (Frame *)scratch_frames.get((uint64_t)(w1 + w2) * depth * sizeof(Frame));
        auto *dq = (DecodeQuery *)dq_buf.get((uint64_t)n * sizeof(DecodeQuery));
        auto *dl = (uint32_t *)dlen_buf.get((uint64_t)n * 8);
        uint32_t *ds = dl + n;
        auto *qn = (DecodeQuery *)hq_buf.get((uint64_t)n * sizeof(DecodeQuery));
        auto *hr = (uint32_t *)hres_buf.get((uint64_t)n * 8);
        std::memcpy(qn, q.data(), (size_t)head * sizeof(DecodeQuery));
        phase.mark("head gathers + launch");
        std::vector<GatherQuery> g1 = take_gathers_pre(qn, 0, head, pg.get());
        auto any_walk = [&](uint32_t lo, uint32_t hi) {
            for (uint32_t j = lo; j < hi; ++j)
                if (qn[j].chunk != kNone) return true;
            return false;
        };
        const bool walk1 = any_walk(0, head);
        if (walk1) hcheck(hipMemcpyAsync(dq, qn, (size_t)head * sizeof(DecodeQuery), hipMemcpyHostToDevice, stream));
        flush_tab();
        hcheck(hipEventRecord(ev0, stream));
        if (walk1)
            hcheck(launch_decode(stream, dq, head, (const RecSlot *const *)chunk_tab, out, dl, ds, frames, depth,
                                 w1 | 0x80000000u, false));
        GatherQuery *dg1 = nullptr, *dg2 = nullptr;
        launch_gathers(stream, g1, out, dl, ds, dg1, 0);
        // the tail: resolved while the head decodes
        phase.mark("tail lookups");
        auto t1 = clk::now();
        parallel_ranges(n - head, host_threads(), [&](uint32_t lo, uint32_t hi) { resolve(head + lo, head + hi); });
        place(head, n);
        lookup_ms = head_ms + std::chrono::duration<double, std::milli>(clk::now() - t1).count();
        if (needed) *needed = total;
        if (total > out_cap) {
            sync();
            release_gathers(dg1);
            return PX_ESPACE;
        }
        phase.mark("tail gathers + launch");
        std::memcpy(qn + head, q.data() + head, (size_t)(n - head) * sizeof(DecodeQuery));
        std::vector<GatherQuery> g2 = take_gathers_pre(qn, head, n, pg.get());
        stats.last_gather_queries = (uint32_t)(g1.size() + g2.size());
        hcheck(hipStreamWaitEvent(stream2, ev0, 0));  // chunk table and head queries uploaded
        if (any_walk(head, n)) {
            hcheck(hipMemcpyAsync(dq + head, qn + head, (size_t)(n - head) * sizeof(DecodeQuery),
                                  hipMemcpyHostToDevice, stream2));
            hcheck(launch_decode(stream2, dq + head, n - head, (const RecSlot *const *)chunk_tab, out, dl + head,
                                 ds + head, frames + (uint64_t)w1 * depth, depth, w2 | 0x80000000u, false));
        }
        launch_gathers(stream2, g2, out, dl + head, ds + head, dg2, 1);
        hcheck(hipEventRecord(ev_join, stream2));
        hcheck(hipStreamWaitEvent(stream, ev_join, 0));
        hcheck(hipEventRecord(ev1, stream));
        phase.mark("sync");
        hcheck(hipMemcpyAsync(hr, dl, (size_t)n * 8, hipMemcpyDeviceToHost, stream));  // lengths, then statuses
        sync();
        phase.mark("results");
        release_gathers(dg1);
        release_gathers(dg2);
        float ms = 0;
        hcheck(hipEventElapsedTime(&ms, ev0, ev1));
        stats.last_decode_kernel_ms = ms;
        for (uint32_t i = 0; i < n; ++i)  // an overrun slot: the plain path re-runs with room (rare)
            if (q[i].chunk != kNone && hr[n + i] == kErrSpace)
                return expand(q, out, out_cap, 1, out_off, out_len, status, needed, pre);
        int rc = PX_OK;
        for (uint32_t i = 0; i < n; ++i) {
            if (q[i].chunk == kNone) {
                out_len[i] = 0;
                status[i] = pre[i];
            } else {
                out_len[i] = hr[i];
                status[i] = map_status(hr[n + i]);
            }
            if (status[i] != PX_OK && rc == PX_OK) rc = (int)status[i];
        }
        return rc;
    }

    // k_link over `jobs` (device copy staged through a scratch buffer)
    void link(const std::vector<LinkJob> &jobs) {
        if (jobs.empty()) return;
        auto *d = (LinkJob *)link_buf.get(jobs.size() * sizeof(LinkJob));
        h2d(d, jobs.data(), jobs.size() * sizeof(LinkJob));
        hcheck(launch_link(stream, (uint32_t)jobs.size(), d));
    }

    // drop every record, keep the device memory for reuse
    void reset() {
        sync();
        dki_clear();
        dki.valid = true;
        for (auto &sp : shards)
            if (sp->arena) heap.release(sp->arena, sp->arena_bytes);
        for (auto &c : chunks)
            if (c.dev) heap.release(c.dev, (uint64_t)c.dev_cap * sizeof(RecSlot));
        for (auto &b : store_blocks)
            if (!arena.owns(b.first)) heap.release(b.first, b.second);
        store_blocks.clear();
        macct = MemAcct{};
        arena.reset();
        last_store = nullptr;
        last_store_bytes = 0;
        shards.clear();
        chunks.clear();
        tab_lo = ~0u;
        tab_hi = 0;
        pending_init.clear();
        pending_state.clear();
        keymap.clear();
        uint64_t held = heap.held();
        stats = px_stats{};
        stats.device_bytes = held;
    }

    int set_batch(uint32_t n, const uint8_t *keys, const uint64_t *koff, const uint8_t *vals,
                  const uint64_t *voff, int on_device, px_set_result *res);
    // stored records whose compat key prefix the CritBit needs (CritBitTree.cpp:27-28)
    struct KpJob {
        uint32_t chunk, idx, doc_len, cap;  // cap: first decode's output cap
    };
    // GPU-decode each record's key prefix (up to the spec-aware 251,0) into its chunk's
    // kp table; a prefix that overran `cap` is decoded again with the whole doc's room.
    // st[i] = kOk or the decode's failure status.
    std::vector<DecodeQuery> kp_queries;
    // set_batch's key-map work, kept across batches: each live key's hash, each partition's records
    std::vector<uint64_t> khash;
    struct KEnt {
        uint64_t h;
        const uint8_t *k;
        uint32_t klen, r, shard, chunk, idx;
    };
    std::vector<KEnt> kents;                          // every partition's entries, partitions in order
    std::array<uint64_t, PartKeyMap::kParts + 1> pstart{};  // partition pi: kents[pstart[pi], pstart[pi + 1])
    void decode_key_prefixes(const std::vector<KpJob> &jobs, std::vector<uint32_t> &st) {
        PhaseClock phase("decode_key_prefixes", "PX_SET_VERBOSE");
        phase.mark("queries");
        st.assign(jobs.size(), kOk);
        const uint32_t nj = (uint32_t)jobs.size();
        // (the query table is kept across batches: value-initialising 40 MB of fresh queries for
        // a million records was most of this phase)
        std::vector<DecodeQuery> &q = kp_queries;
        q.resize(nj);
        std::vector<uint32_t> qj(nj);
        std::vector<uint64_t> qoff(nj + 1);
        pxh::parallel_prefix(nj, nj >= 65536 ? host_threads() : 1, qoff.data(),
                             [&](uint32_t i) -> uint64_t { return round_up(jobs[i].cap, 16); });
        parallel_ranges(nj, nj >= 65536 ? host_threads() : 1, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t i = lo; i < hi; ++i) {
                q[i] = DecodeQuery{jobs[i].chunk, jobs[i].idx, 0, kMaxDoc, qoff[i], jobs[i].cap, 0};
                qj[i] = i;
            }
        });
        uint64_t qo = qoff[nj];
        for (int pass = 0; pass < 2 && !q.empty(); ++pass) {
            phase.mark(pass ? "decode (again)" : "decode");
            auto *kbuf = (uint8_t *)heap.alloc(qo + 64);
            std::vector<uint32_t> ql, qs;
            run_decode(q, kbuf, ql, qs, false);
            phase.mark("copy down");
            // (through a pinned buffer kept across batches: a million key prefixes are ~60 MB,
            // which a pageable copy moved at a fifth of the rate)
            auto *hk = (uint8_t *)kp_hbuf.get(qo + 1);
            hcheck(hipMemcpyAsync(hk, kbuf, qo, hipMemcpyDeviceToHost, stream));
            sync();
            heap.release(kbuf, qo + 64);
            phase.mark("append to the chunks' prefix stores");
            std::vector<DecodeQuery> again;
            std::vector<uint32_t> again_j;
            uint64_t ao = 0;
            // the first pass's overruns go again with room; everything else is appended to
            // its chunk's prefix store, chunks in parallel (a chunk's queries are contiguous)
            std::vector<uint8_t> redo(q.size(), 0);
            // (failures and overruns marked on host threads; the few overruns collected in order)
            parallel_ranges((uint32_t)q.size(), q.size() >= 65536 ? host_threads() : 1, [&](uint32_t lo, uint32_t hi) {
                for (uint32_t i = lo; i < hi; ++i) {
                    if (qs[i] != kOk && qs[i] != kErrSpace) {
                        st[qj[i]] = qs[i];
                        redo[i] = 2;
                    } else if (pass == 0 && qs[i] == kErrSpace && key_end(hk + q[i].out_off, ql[i]) == 0) {
                        redo[i] = 1;
                    }
                }
            });
            for (size_t i = 0; i < q.size(); ++i) {
                if (redo[i] == 1) {
                    DecodeQuery d = q[i];
                    d.out_off = ao;
                    d.out_cap = jobs[qj[i]].doc_len + 256;
                    ao += round_up(d.out_cap, 16);
                    again.push_back(d);
                    again_j.push_back(qj[i]);
                }
            }
            std::vector<uint32_t> runs;  // [runs[k], runs[k+1]): one chunk's queries
            for (uint32_t i = 0; i < (uint32_t)q.size(); ++i)
                if (i == 0 || q[i].chunk != q[i - 1].chunk) runs.push_back(i);
            runs.push_back((uint32_t)q.size());
            auto append_run = [&](uint32_t k) {
                for (uint32_t i = runs[k]; i < runs[k + 1]; ++i) {
                    if (redo[i]) continue;
                    const KpJob &j = jobs[qj[i]];
                    const uint8_t *p = hk + q[i].out_off;
                    const uint32_t ke = key_end(p, ql[i]);
                    const uint32_t keep = ke ? ke : ql[i];
                    Chunk &ch = chunks[j.chunk];
                    ch.kp_off[j.idx] = ch.kp.size();
                    ch.kp_len[j.idx] = keep;
                    ch.kp.append(reinterpret_cast<const char *>(p), keep);
                }
            };
            bool distinct = true;  // a chunk in two runs (possible in the second pass): in order
            {
                std::unordered_set<uint32_t> seen;
                for (uint32_t k = 0; k + 1 < runs.size() && distinct; ++k) distinct = seen.insert(q[runs[k]].chunk).second;
            }
            if (distinct && runs.size() > 2 && q.size() >= 4096) {
                const std::function<void(uint32_t)> job = [&](uint32_t k) { append_run(k); };
                WorkerPool::get().run((uint32_t)runs.size() - 1, job);
            } else {
                for (uint32_t k = 0; k + 1 < runs.size(); ++k) append_run(k);
            }
            q.assign(again.begin(), again.end());
            qj.swap(again_j);
            qo = ao;
        }
    }
    // PiXiuCtrl-level setitem / delitem with the reinsert compaction (PiXiuCtrl.cpp:12-29,
    // 63-69, 88-114); set_batch is the batch SuffixTree::setitem + CritBit underneath
    bool raw_docs = false;  // set_batch input is ready docs (reinserted records)
    int set_ctrl(uint32_t n, const uint8_t *keys, const uint64_t *koff, const uint8_t *vals, const uint64_t *voff,
                 int on_device, px_set_result *res);
    void reinsert_chunk(Shard &s, uint32_t c, bool via_glob);
    enum { kTrigSet, kTrigReinsert, kTrigDel };
    void reinsert_triggers(Shard &s, int when);
    int del_ctrl(uint32_t n, const uint8_t *keys, const uint64_t *koff, uint32_t *result);
    // chunk blob (include/pixiu_amd.h: px_save / px_load)
    int save(uint8_t *dst, uint64_t cap, int dst_on_device, uint64_t *bytes);
    int load(const uint8_t *src, uint64_t len, int src_on_device, uint32_t *first_shard);
    // PX_DEBUG_POISON=1: fill the batch scratch with garbage before each set batch (tests
    // that no per-record result depends on what an earlier batch left there)
    static bool debug_poison() {
        const char *e = test_hook("PX_DEBUG_POISON");
        return e && *e && *e != '0';
    }
    ~px_ctx() {
        for (auto &b : pin_blocks) (void)hipHostFree(b.first);
    }
    int expand(const std::vector<DecodeQuery> &q0, uint8_t *out, uint64_t out_cap, int out_on_device,
               uint64_t *out_off, uint32_t *out_len, uint32_t *status, uint64_t *needed,
               const std::vector<uint32_t> &pre_status);
};

namespace {
px_status map_status(uint32_t s) {
    switch (s) {
    case kOk: return PX_OK;
    case kErrInval: return PX_EINVAL;
    case kErrCapacity: return PX_ECAPACITY;
    case kErrRefCrash: return PX_EREFCRASH;
    case kErrCorrupt: return PX_ECORRUPT;
    case kErrHang: return PX_EHANG;
    case kErrDepth: return PX_EDEPTH;
    case kErrSpace: return PX_ESPACE;
    default: return PX_ECORRUPT;
    }
}

// first spec-aware 251,0 in a decoded stream: returns prefix length incl. it, or 0
uint32_t key_end(const uint8_t *p, uint32_t n) {
    bool spec = false;
    for (uint32_t k = 0; k < n; ++k) {
        if (!spec && p[k] == kEsc) {
            spec = true;
        } else if (spec) {
            if (p[k] == kKeyEnd) return k + 1;
            spec = false;
        }
    }
    return 0;
}
}  // namespace

std::string px_ctx::crit_key(const uint8_t *k, uint64_t n) const {
    if (!raw_docs) return esc_key(k, n);
    return std::string(reinterpret_cast<const char *>(k), key_end(k, (uint32_t)n));
}

int px_ctx::set_batch(uint32_t n, const uint8_t *keys, const uint64_t *koff, const uint8_t *vals,
                      const uint64_t *voff, int on_device, px_set_result *res) {
    if (n == 0) return PX_OK;
    // A shard's text is addressed with 32-bit offsets from its live chunk (buffer
    // resources of 2^31 bytes): a batch that could put more than kMaxBatchRaw raw
    // bytes (<= 2x that escaped) into one shard is processed in pieces, in order --
    // the same records in the same order, so the same result.
    if (n > 1 && (opts.records_per_shard == 0 || opts.records_per_shard > 4096)) {
        std::vector<uint64_t> ko(n + 1), vo(n + 1);
        if (on_device) {
            d2h(ko.data(), koff, (size_t)(n + 1) * 8);
            d2h(vo.data(), voff, (size_t)(n + 1) * 8);
            sync();
        } else {
            std::memcpy(ko.data(), koff, (size_t)(n + 1) * 8);
            std::memcpy(vo.data(), voff, (size_t)(n + 1) * 8);
        }
        if ((ko[n] - ko[0]) + (vo[n] - vo[0]) > kMaxBatchRaw) {
            int rc = PX_OK;
            px_stats acc{};  // the batch's timings: the pieces' sums
            for (uint32_t a = 0; a < n;) {
                uint32_t b = a + 1;
                while (b < n && (ko[b + 1] - ko[a]) + (vo[b + 1] - vo[a]) <= kMaxBatchRaw) ++b;
                const int r2 = set_batch(b - a, keys, koff + a, vals, voff + a, on_device, res ? res + a : nullptr);
                if (rc == PX_OK) rc = r2;
                acc.last_set_stage_ms += stats.last_set_stage_ms;
                acc.last_encode_stage_ms += stats.last_encode_stage_ms;
                acc.last_emit_kernel_ms += stats.last_emit_kernel_ms;
                acc.last_psa_ms += stats.last_psa_ms;
                acc.last_psa_sort_ms += stats.last_psa_sort_ms;
                acc.last_psa_lcp_ms += stats.last_psa_lcp_ms;
                acc.last_psa_msg_ms += stats.last_psa_msg_ms;
                acc.last_psa_pool_ms += stats.last_psa_pool_ms;
                acc.last_psa_rounds += stats.last_psa_rounds;
                acc.last_psa_rotations += stats.last_psa_rotations;
                acc.last_span_build_ms += stats.last_span_build_ms;
                acc.last_psa_shards = std::max(acc.last_psa_shards, stats.last_psa_shards);
                acc.last_walk_shards = std::max(acc.last_walk_shards, stats.last_walk_shards);
                acc.last_psa_iters = std::max(acc.last_psa_iters, stats.last_psa_iters);
                acc.last_set_peak_bytes = std::max(acc.last_set_peak_bytes, stats.last_set_peak_bytes);
                a = b;
            }
            stats.last_set_stage_ms = acc.last_set_stage_ms;
            stats.last_encode_stage_ms = acc.last_encode_stage_ms;
            stats.last_emit_kernel_ms = acc.last_emit_kernel_ms;
            stats.last_psa_ms = acc.last_psa_ms;
            stats.last_psa_sort_ms = acc.last_psa_sort_ms;
            stats.last_psa_lcp_ms = acc.last_psa_lcp_ms;
            stats.last_psa_msg_ms = acc.last_psa_msg_ms;
            stats.last_psa_pool_ms = acc.last_psa_pool_ms;
            stats.last_psa_rounds = acc.last_psa_rounds;
            stats.last_psa_rotations = acc.last_psa_rotations;
            stats.last_span_build_ms = acc.last_span_build_ms;
            stats.last_psa_shards = acc.last_psa_shards;
            stats.last_walk_shards = acc.last_walk_shards;
            stats.last_psa_iters = acc.last_psa_iters;
            stats.last_set_peak_bytes = acc.last_set_peak_bytes;
            return rc;
        }
    }
    PhaseClock phase("set_batch", "PX_SET_VERBOSE");
    if (test_hook("PX_DEBUG_SET_THROW")) throw std::bad_alloc();  // (test hook: a failing batch)
    heap.mark_peak();  // (this batch's scratch peak: trim_heap keeps that much cached)
    phase.mark("inputs on device; raw keys also on host ");
    // ---- inputs on device; raw keys also on host (the CritBit needs them)
    std::vector<uint64_t> hkoff(n + 1), hvoff(n + 1);
    const uint8_t *dkeys, *dvals;
    const uint64_t *dkoff, *dvoff;
    std::vector<uint8_t> hkeys;
    if (on_device) {
        d2h(hkoff.data(), koff, (n + 1) * 8);
        d2h(hvoff.data(), voff, (n + 1) * 8);
        sync();
        hkeys.resize(hkoff[n] - hkoff[0]);
        d2h(hkeys.data(), keys + hkoff[0], hkeys.size());
        sync();
        // (rebase by a copy: hkoff[0] itself becomes 0 on the first iteration)
        const uint64_t k0 = hkoff[0];
        for (auto &o : hkoff) o -= k0;
        dkeys = keys;
        dvals = vals;
        dkoff = koff;
        dvoff = voff;
        // (device koff may not start at 0: the kernels use absolute offsets)
    } else {
        memcpy(hkoff.data(), koff, (n + 1) * 8);
        memcpy(hvoff.data(), voff, (n + 1) * 8);
        uint64_t kb = koff[n] - koff[0], vb = voff[n] - voff[0];
        hkeys.assign(keys + koff[0], keys + koff[n]);
        uint64_t tot = kb + vb + (n + 1) * 16 + 512;
        auto *b = (uint8_t *)in_buf.get(tot);
        auto *dk = b;
        auto *dv = b + round_up(kb, 64);
        auto *dko = (uint64_t *)(dv + round_up(vb, 64));
        auto *dvo = dko + (n + 1);
        h2d_bulk(dk, keys + koff[0], kb);
        h2d_bulk(dv, vals + voff[0], vb);
        std::vector<uint64_t> k0(n + 1), v0(n + 1);
        for (uint32_t i = 0; i <= n; ++i) {
            k0[i] = koff[i] - koff[0];
            v0[i] = voff[i] - voff[0];
        }
        h2d(dko, k0.data(), (n + 1) * 8);
        h2d(dvo, v0.data(), (n + 1) * 8);
        for (auto &o : hkoff) o -= koff[0];
        for (auto &o : hvoff) o -= voff[0];
        dkeys = dk;
        dvals = dv;
        dkoff = dko;
        dvoff = dvo;
    }

    phase.mark("pass 1: escaped doc lengths");
    // ---- pass 1: escaped doc lengths
    auto *tmp = (uint32_t *)tmp_buf.get((uint64_t)n * 28 + 64);
    uint32_t *d_doclen = tmp, *d_complen = tmp + n, *d_chunk = tmp + 2 * n, *d_idx = tmp + 3 * n,
             *d_status = tmp + 4 * n, *d_nseg = tmp + 5 * n, *d_nesc = tmp + 6 * n;
    if (debug_poison()) hcheck(hipMemsetAsync(tmp, 0xa5, (size_t)n * 28 + 64, stream));  // stale-scratch test
    hcheck(launch_doc_len(stream, n, dkeys, dkoff, raw_docs ? nullptr : dvals, dvoff, d_doclen, d_complen));
    std::vector<uint32_t> doc_len(n);
    d2h(doc_len.data(), d_doclen, n * 4);
    sync();

    phase.mark("shard assignment: contiguous, in arrival");
    // ---- shard assignment: contiguous, in arrival order
    std::vector<uint32_t> rec_shard(n);
    struct Work {
        Shard *s;
        uint32_t r0, r1;
        uint64_t bytes;
        uint32_t docs;
    };
    std::vector<Work> work;
    for (uint32_t r = 0; r < n; ++r) {
        Shard *s;
        if (opts.records_per_shard == 0) {
            s = shards.empty() ? &new_shard() : shards[0].get();
        } else {
            s = shards.empty() ? &new_shard() : shards.back().get();
            if (s->records >= opts.records_per_shard) s = &new_shard();
        }
        s->records++;
        rec_shard[r] = s->id;
        if (work.empty() || work.back().s != s) work.push_back(Work{s, r, r, 0, 0});
        work.back().r1 = r + 1;
        if (doc_len[r] != 0xffffffffu) {
            work.back().bytes += doc_len[r];
            work.back().docs++;
        }
    }
    for (const Work &w : work)  // a live chunk + batch beyond 32-bit text offsets (pathological)
        if (w.s->text_end - w.s->hs.ctext_off + w.bytes > kMaxShardText) {
            for (const Work &u : work) u.s->records -= u.r1 - u.r0;
            return PX_ECAPACITY;
        }

    phase.mark("which shards take the suffix-array path ");
    // ---- which shards take the suffix-array path (px_psa.hip)
    // A PSA live chunk never has a suffix tree.  One whose stream the PSA check flags goes
    // to k_gst_encode, which first re-walks (replays) the docs PSA encoded.
    const bool psa_on = psa_enabled();
    // a PSA live chunk that is slot-full rotates at this batch's first doc (PiXiuCtrl.cpp:13):
    // the new chunk starts empty, so the rotation is done here and the batch stays on PSA
    for (const Work &w : work) {
        Shard &sh = *w.s;
        if (sh.psa && w.docs > 0 && sh.hs.n_docs == (uint32_t)kChunkSlots) {
            sh.hs.chunk_seq++;
            sh.hs.n_docs = 0;
            sh.hs.ctext_off = 0;
            sh.text_end = 0;
        }
    }
    // A live chunk is encoded by PSA unless it already has a suffix tree (a walked chunk).
    // Where the live chunk could rotate inside the batch (more than kPsaMaxText doc bytes),
    // the MemPool accounting is emulated on the suffix array (k_pool_*) and the docs after a
    // rotation go to the next chunk in another round.
    std::vector<uint8_t> wpsa(work.size(), 0);
    std::vector<uint32_t> wreplay(work.size(), 0), wr0(work.size());
    for (size_t k = 0; k < work.size(); ++k) {
        const Work &w = work[k];
        const Shard &sh = *w.s;
        const bool fresh = sh.psa || (sh.hs.epoch == 0 && sh.hs.n_docs == 0);
        wpsa[k] = psa_on && fresh && w.docs > 0;
        wr0[k] = w.r0;
    }

    phase.mark("arenas, doc destinations, comp scratch");
    // ---- arenas, doc destinations, comp scratch
    // (both tables in pinned memory kept across batches, copied to the device from there)
    auto **dst = static_cast<uint8_t **>(dst_pin.get((uint64_t)n * 16 + 64)), **cdst = dst + n;
    uint64_t scratch_bytes = 0;
    for (uint32_t r = 0; r < n; ++r)
        if (doc_len[r] != 0xffffffffu) scratch_bytes += round_up(doc_len[r], 16);
    auto *comp_scratch = (uint8_t *)heap.alloc(scratch_bytes + 256);
    // encoder messages: one u32 per doc byte, at 4x the record's comp scratch offset
    auto *msgs = (uint32_t *)heap.alloc(scratch_bytes * 4 + 256);
    uint64_t so = 0;
    for (size_t k = 0; k < work.size(); ++k) {
        Work &w = work[k];
        if (wpsa[k]) text_reserve(*w.s, w.bytes);
        else if (w.s->text_only) wreplay[k] = upgrade_to_walk(*w.s, w.bytes, w.docs);
        else shard_reserve(*w.s, w.bytes, w.docs);
        uint64_t t = w.s->text_end;
        for (uint32_t r = w.r0; r < w.r1; ++r) {
            if (doc_len[r] == 0xffffffffu) {
                dst[r] = cdst[r] = nullptr;
                continue;
            }
            dst[r] = w.s->text + t;
            t += doc_len[r];
            cdst[r] = comp_scratch + so;
            so += round_up(doc_len[r], 16);
        }
        w.s->text_end = t;
    }
    auto *d_dst = (uint8_t **)heap.alloc((uint64_t)n * 8);
    auto *d_cdst = (uint8_t **)heap.alloc((uint64_t)n * 8);
    hcheck(hipMemcpyAsync(d_dst, dst, (size_t)n * 8, hipMemcpyHostToDevice, stream));
    hcheck(hipMemcpyAsync(d_cdst, cdst, (size_t)n * 8, hipMemcpyHostToDevice, stream));
    flush_shard_init();
    hcheck(launch_doc_write(stream, n, dkeys, dkoff, raw_docs ? nullptr : dvals, dvoff, d_dst));

    phase.mark("the suffix-array path over the PSA shard");
    // ---- the suffix-array path over the PSA shards (messages, placement, check flags), in
    // rounds: a round takes every unfinished shard's live chunk plus a window of its next
    // docs; a shard whose live chunk rotates inside the window keeps the docs before the
    // rotation and starts the next round with an empty chunk
    hcheck(hipEventRecord(ev0, stream));
    uint32_t psa_shards = 0, walk_shards = 0, psa_rounds = 0, psa_rotations = 0;
    double psa_ms = 0;
    {
        struct Run {
            size_t k;
            std::vector<uint32_t> recs;  // valid records, in order
            size_t next = 0;             // first record not placed yet
            uint32_t seq = 0;
            std::vector<std::pair<const uint8_t *, uint32_t>> live;  // live chunk docs
            uint64_t live_bytes = 0, live_off = 0;
            uint64_t window = 0;  // new doc bytes per round while the chunk may rotate
            bool done = false;
        };
        std::vector<Run> runs;
        const uint64_t win0 = [] {
            const char *e = std::getenv("PX_PSA_WINDOW_MB");
            return (uint64_t)((e ? std::atof(e) : 12.0) * 1048576.0);
        }();
        for (size_t k = 0; k < work.size(); ++k) {
            if (!wpsa[k]) continue;
            const Work &w = work[k];
            Shard &sh = *w.s;
            Run u;
            u.k = k;
            u.seq = sh.hs.chunk_seq;
            for (uint32_t r = w.r0; r < w.r1; ++r)
                if (doc_len[r] != 0xffffffffu) u.recs.push_back(r);
            if (sh.psa && sh.hs.n_docs) {  // the live chunk's earlier docs (text_reserve put them at 0)
                const Chunk &ch = chunks[sh.chunks[sh.hs.chunk_seq]];
                for (uint32_t i = 0; i < sh.hs.n_docs; ++i) {
                    u.live.emplace_back(sh.text + u.live_bytes, ch.doc_len[i]);
                    u.live_bytes += ch.doc_len[i];
                }
            }
            u.window = win0;
            runs.push_back(std::move(u));
        }
        auto *d_pool = (PsaPoolOut *)heap.alloc(std::max<size_t>(runs.size(), 1) * sizeof(PsaPoolOut) + 64);
        const auto tp = std::chrono::steady_clock::now();
        PsaStats pst{};
        for (;;) {
            std::vector<PsaDoc> pd;
            std::vector<PsaShard> ps;
            std::vector<size_t> prun;
            std::vector<uint32_t> pcount;  // new docs in the window
            uint64_t gpos = 0;
            bool any_pools = false;
            // a round holds at most round_cap positions (device scratch, 32-bit positions)
            // and kPsaMaxShards shards (the first sort key's shard bits); the shards that do
            // not fit wait for the next round
            const uint64_t round_cap = psa_round_cap();
            for (size_t ri = 0; ri < runs.size(); ++ri) {
                Run &u = runs[ri];
                if (u.done) continue;
                if (ps.size() >= kPsaMaxShards) break;
                Shard &sh = *work[u.k].s;
                if (u.live.size() == (size_t)kChunkSlots) {  // slot-full: rotation before the next doc
                    ++u.seq;
                    ++psa_rotations;
                    u.live.clear();
                    u.live_bytes = 0;
                    u.live_off = (uint64_t)(dst[u.recs[u.next]] - sh.text);
                }
                const uint32_t si = (uint32_t)ps.size();
                PsaShard psh{};
                psh.base = (uint32_t)gpos;
                psh.chunk = u.seq;
                psh.doc0 = (uint32_t)pd.size();
                uint64_t off = 0;
                uint32_t slot = 0;
                for (const auto &lv : u.live) {
                    pd.push_back(PsaDoc{lv.first, nullptr, (uint32_t)(gpos + off), lv.second, si, slot++, 0, 0});
                    off += lv.second;
                }
                // the window: every remaining doc if the chunk cannot rotate on them,
                // else up to u.window new bytes (at least one doc)
                uint64_t rest = 0;
                for (size_t i = u.next; i < u.recs.size(); ++i) rest += doc_len[u.recs[i]];
                const bool may_rotate = u.live_bytes + rest > kPsaMaxText;
                // (new bytes: up to the window, and at least half a window once the live
                // chunk alone has outgrown it without rotating)
                const uint64_t win = std::max<uint64_t>(u.window, kPsaMaxText);
                // (and no more than the round's position cap leaves: a chunk that does not
                // rotate inside a shorter window simply continues in the next round)
                const uint64_t room = round_cap > gpos + u.live_bytes ? round_cap - gpos - u.live_bytes : 0;
                const uint64_t budget =
                    std::min(std::max<uint64_t>(win > u.live_bytes ? win - u.live_bytes : 0, win / 2), room);
                uint32_t cnt = 0;
                uint64_t nb = 0;
                for (size_t i = u.next; i < u.recs.size() && u.live.size() + cnt < (size_t)kChunkSlots; ++i) {
                    const uint32_t r = u.recs[i];
                    if (may_rotate && cnt > 0 && nb + doc_len[r] > budget) break;
                    pd.push_back(PsaDoc{dst[r], msgs + (cdst[r] - comp_scratch), (uint32_t)(gpos + off), doc_len[r], si,
                                        slot++, r, 0});
                    off += doc_len[r];
                    nb += doc_len[r];
                    ++cnt;
                }
                if (!ps.empty() && gpos + off > round_cap) {  // (a round takes at least one shard)
                    pd.resize(psh.doc0);
                    break;
                }
                psh.len = (uint32_t)off;
                psh.ndocs = (uint32_t)(pd.size() - psh.doc0);
                psh.pools = u.live_bytes + nb > kPsaMaxText ? 1u : 0u;
                any_pools |= psh.pools != 0;
                ps.push_back(psh);
                prun.push_back(ri);
                pcount.push_back(cnt);
                gpos += off;
            }
            if (ps.empty()) break;
            ++psa_rounds;
            if (gpos >= 0xfffffff0ull) throw PxFail{PX_ECAPACITY};  // a batch is split far below this
            auto *d_pd = (PsaDoc *)heap.alloc(pd.size() * sizeof(PsaDoc));
            auto *d_ps = (PsaShard *)heap.alloc(ps.size() * sizeof(PsaShard) + ps.size() * 4 + 64);
            auto *d_flag = (uint32_t *)(d_ps + ps.size());
            h2d(d_pd, pd.data(), pd.size() * sizeof(PsaDoc));
            h2d(d_ps, ps.data(), ps.size() * sizeof(PsaShard));
            hcheck(hipMemsetAsync(d_flag, 0, ps.size() * 4, stream));
            PsaAlloc A{[](void *self, uint64_t b) { return static_cast<px_ctx *>(self)->heap.alloc(b); },
                       [](void *self, void *p, uint64_t b) { static_cast<px_ctx *>(self)->heap.release(p, b); }, this,
                       static_cast<uint32_t *>(psa_pin.get(kPsaPinWords * 4))};
            PsaStats rst{};
            hcheck(psa_run(stream, A, (uint32_t)pd.size(), d_pd, (uint32_t)ps.size(), d_ps, ps.data(), (uint32_t)gpos, d_chunk,
                           d_idx, d_status, d_flag, any_pools, d_pool, &rst));
            std::vector<uint32_t> flag(ps.size());
            std::vector<PsaPoolOut> pout(ps.size());
            d2h(flag.data(), d_flag, ps.size() * 4);
            if (any_pools) d2h(pout.data(), d_pool, ps.size() * sizeof(PsaPoolOut));
            sync();
            if (const char *e = std::getenv("PX_DEBUG_PSA_FLAG_ROUND"))  // test hook: the check fires
                if ((uint32_t)std::atoi(e) == psa_rounds) std::fill(flag.begin(), flag.end(), 1u);
            if (!any_pools) rst.ms_pool = 0.f;
            if (psa_rounds == 1) {
                pst = rst;
            } else {
                pst.ms_sort += rst.ms_sort;
                pst.ms_lcp += rst.ms_lcp;
                pst.ms_msg += rst.ms_msg;
                pst.ms_pool += rst.ms_pool;
                pst.candidates += rst.candidates;
                pst.iterations = std::max(pst.iterations, rst.iterations);
            }
            if (const char *v = std::getenv("PX_PSA_VERBOSE"); v && *v == '1') {
                uint32_t nf = 0, nr = 0, nb = 0;
                for (size_t i = 0; i < ps.size(); ++i) {
                    nf += flag[i] != 0;
                    nr += ps[i].pools && pout[i].rot_doc != kNone;
                    nb += ps[i].pools && pout[i].how != 0;
                }
                fprintf(stderr, "psa round %u: %zu shards, %zu docs, N=%llu, pools %d (%u candidates, %.2f ms, "
                                "%u decided by the bound), %u rotations, %u flagged, sort %.2f lcp %.2f msg %.2f ms\n",
                        psa_rounds, ps.size(), pd.size(), (unsigned long long)gpos, (int)any_pools, rst.candidates,
                        rst.ms_pool, nb, nr, nf, rst.ms_sort, rst.ms_lcp, rst.ms_msg);
            }
            heap.release(d_pd, pd.size() * sizeof(PsaDoc));
            heap.release(d_ps, ps.size() * sizeof(PsaShard) + ps.size() * 4 + 64);
            for (size_t i = 0; i < ps.size(); ++i) {
                Run &u = runs[prun[i]];
                Shard &sh = *work[u.k].s;
                if (ps[i].pools && pout[i].how == 3) {  // (k_pool_scan reached no verdict: cannot happen)
                    fprintf(stderr, "pixiu_amd: MemPool emulation stalled on shard %u; walking it\n", sh.id);
                    flag[i] = 1;
                }
                if (flag[i]) {
                    // the stale-pair check fired: this shard's live chunk and its remaining docs
                    // go to the walk (the text copied includes them; their records keep reading
                    // their docs from the old arena, released at the end of the batch)
                    std::vector<uint32_t> lens;
                    for (const auto &lv : u.live) lens.push_back(lv.second);
                    sh.hs.chunk_seq = u.seq;
                    wpsa[u.k] = 0;
                    wr0[u.k] = u.recs[u.next];
                    wreplay[u.k] = upgrade_to_walk(sh, 0, (uint32_t)(u.recs.size() - u.next), u.live_off, lens);
                    u.done = true;
                    continue;
                }
                const uint32_t first_new = ps[i].doc0 + (uint32_t)u.live.size();
                const bool rot = ps[i].pools && pout[i].rot_doc != kNone;
                const uint32_t take = rot ? pout[i].rot_doc - first_new : pcount[i];
                uint64_t took = 0;
                for (uint32_t t = 0; t < take; ++t) {
                    const uint32_t r = u.recs[u.next + t];
                    u.live.emplace_back(dst[r], doc_len[r]);
                    took += doc_len[r];
                }
                u.live_bytes += took;
                u.next += take;
                if (rot) {
                    // the window for the next chunk: a little more than this one held (chunks of
                    // one corpus hold nearly the same bytes: config 3's 51 full chunks are
                    // 194-196 docs; a window that misses costs one more round for that chunk)
                    u.window = std::max<uint64_t>(kPsaMaxText, u.live_bytes + u.live_bytes / 40);
                    ++u.seq;
                    ++psa_rotations;
                    u.live.clear();
                    u.live_bytes = 0;
                    u.live_off = u.next < u.recs.size() ? (uint64_t)(dst[u.recs[u.next]] - sh.text) : sh.text_end;
                }
                if (u.next >= u.recs.size()) {
                    u.done = true;
                    ++psa_shards;
                    sh.psa = true;
                    sh.hs.n_docs = (uint32_t)u.live.size();
                    sh.hs.chunk_seq = u.seq;
                    sh.hs.ctext_off = u.live_off;
                }
            }
            flush_shard_init();
        }
        heap.release(d_pool, std::max<size_t>(runs.size(), 1) * sizeof(PsaPoolOut) + 64);
        psa_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count();
        psa_stats = pst;
    }

    phase.mark("the GST walk for the other shards (encod");
    // ---- the GST walk for the other shards (encoder messages)
    std::vector<GstShard> gs;
    std::vector<size_t> gwork;
    for (size_t k = 0; k < work.size(); ++k) {
        if (wpsa[k]) continue;
        const Work &w = work[k];
        GstShard g{};
        g.text = w.s->text;
        g.doc_base = w.s->doc_base;
        g.nodes = w.s->nodes;
        g.hash = w.s->hash;
        g.root = w.s->root_tab;
        g.st = w.s->st;
        g.node_cap = w.s->node_cap;
        g.hash_mask = (uint32_t)(w.s->hash_cap - 1);
        g.doc_cap = w.s->doc_cap;
        g.r0 = wr0[k];
        g.r1 = w.r1;
        g.replay = wreplay[k];
        gs.push_back(g);
        gwork.push_back(k);
    }
    walk_shards = (uint32_t)gs.size();
    GstShard *d_gs = nullptr;
    auto *d_stout = (ShardState *)stout_buf.get(std::max<size_t>(gs.size(), 1) * sizeof(ShardState));
    if (!gs.empty()) {
        d_gs = (GstShard *)heap.alloc(gs.size() * sizeof(GstShard));
        h2d(d_gs, gs.data(), gs.size() * sizeof(GstShard));
        auto *sink = (uint32_t *)sink_buf.get((uint64_t)(kMaxDoc + 64) * 4);
        hcheck(launch_gst_encode(stream, d_gs, (uint32_t)gs.size(), d_doclen, d_cdst, comp_scratch, msgs, d_chunk,
                                 d_idx, d_status, d_stout, sink));
    }
    hcheck(hipEventRecord(ev_mid, stream));
    // the encoder's record tokens (k_tok_segs builds the segment index from them): room for
    // doc_len / 7 + 2 per record (a token stands for a run of 7 or more doc bytes)
    std::vector<uint64_t> tok_off(n + 1);
    pxh::parallel_prefix(n, n >= 65536 ? host_threads() : 1, tok_off.data(),
                         [&](uint32_t r) -> uint64_t { return doc_len[r] == 0xffffffffu ? 0 : doc_len[r] / 7 + 2; });
    const uint64_t tok_n = tok_off[n];
    auto *d_toks = (TokEnt *)heap.alloc(tok_n * sizeof(TokEnt) + 64);
    auto *d_tokoff = (uint64_t *)heap.alloc((uint64_t)n * 12 + 64);
    auto *d_ntok = (uint32_t *)(d_tokoff + n);
    h2d(d_tokoff, tok_off.data(), (size_t)n * 8);
    hcheck(launch_gst_emit(stream, n, d_dst, d_doclen, d_cdst, comp_scratch, msgs, d_status, d_complen, d_tokoff, d_toks,
                           d_ntok));
    hcheck(hipEventRecord(ev1, stream));
    hcheck(launch_count_esc(stream, n, d_cdst, d_complen, d_nesc));
    std::vector<uint32_t> comp_len(n), rchunk(n), ridx(n), rstatus(n), nesc(n), ntok(n);
    d2h(nesc.data(), d_nesc, n * 4);
    d2h(ntok.data(), d_ntok, n * 4);  // (sizes the segment index: k_tok_segs writes 2 ntok + 2 entries at most)
    d2h(comp_len.data(), d_complen, n * 4);
    d2h(rchunk.data(), d_chunk, n * 4);
    d2h(ridx.data(), d_idx, n * 4);
    d2h(rstatus.data(), d_status, n * 4);
    std::vector<ShardState> stout(gs.size());
    if (!gs.empty()) d2h(stout.data(), d_stout, gs.size() * sizeof(ShardState));
    sync();
    // Invariants of the walk + encoder: a record the walk placed (chunk/slot written)
    // has a compressed form of 1..2*doc_len+8 bytes; a record it did not place has a
    // non-OK status.  Every word was defined by k_doc_len for this batch, so a
    // violation is a kernel or transfer bug: fail loudly, never repair.
    int corrupt = 0;
    // (the check on host threads for big batches; a range with a violation is re-run in order
    // below so the messages and repairs come out as the serial loop made them)
    std::atomic<bool> any_bad{false};
    if (n >= 65536) {
        parallel_ranges(n, host_threads(), [&](uint32_t lo, uint32_t hi) {
            bool b = false;
            for (uint32_t r = lo; r < hi && !b; ++r) {
                const bool valid = doc_len[r] != 0xffffffffu;
                const bool pl = rchunk[r] != 0xffffffffu && ridx[r] != 0xffffffffu;
                b = pl ? (!valid || comp_len[r] == 0 || comp_len[r] > 2 * doc_len[r] + 8 || rstatus[r] > kErrSpace)
                       : (rstatus[r] == kOk || (valid && rstatus[r] > kErrSpace));
            }
            if (b) any_bad.store(true);
        });
    }
    for (uint32_t r = 0; r < (n < 65536 || any_bad.load() ? n : 0u); ++r) {
        const bool valid = doc_len[r] != 0xffffffffu;
        const bool placed = rchunk[r] != 0xffffffffu && ridx[r] != 0xffffffffu;
        bool bad = false;
        if (placed) bad = !valid || comp_len[r] == 0 || comp_len[r] > 2 * doc_len[r] + 8 || rstatus[r] > kErrSpace;
        else bad = rstatus[r] == kOk || (valid && rstatus[r] > kErrSpace);
        if (bad) {
            fprintf(stderr, "pixiu_amd: internal error: record %u of a %u-record batch: doc %u B, placed %d "
                            "(chunk %u slot %u), status %u, comp_len %u\n",
                    r, n, doc_len[r], (int)placed, rchunk[r], ridx[r], rstatus[r], comp_len[r]);
            if (!placed) rstatus[r] = kErrCorrupt;
            else if (rstatus[r] == kOk) rstatus[r] = kErrCorrupt;
            corrupt = PX_ECORRUPT;
        }
    }
    if (const char *e = test_hook("PX_DEBUG_FAIL_REC")) {  // test hook: fail one placed record
        const uint32_t r = (uint32_t)std::atoi(e);
        if (r < n && rstatus[r] == kOk) rstatus[r] = kErrCorrupt;
    }
    for (size_t i = 0; i < gwork.size(); ++i) work[gwork[i]].s->hs = stout[i];
    stats.last_psa_ms = psa_ms;
    stats.last_psa_sort_ms = psa_shards ? psa_stats.ms_sort : 0;
    stats.last_psa_lcp_ms = psa_shards ? psa_stats.ms_lcp : 0;
    stats.last_psa_msg_ms = psa_shards ? psa_stats.ms_msg : 0;
    stats.last_psa_iters = psa_shards ? psa_stats.iterations : 0;
    stats.last_psa_shards = psa_shards;
    stats.last_psa_rounds = psa_rounds;
    stats.last_psa_rotations = psa_rotations;
    stats.last_psa_pool_ms = psa_shards ? psa_stats.ms_pool : 0;
    stats.last_walk_shards = walk_shards;
    if (d_gs) heap.release(d_gs, gs.size() * sizeof(GstShard));
    {
        float ms = 0;
        hcheck(hipEventElapsedTime(&ms, ev0, ev1));
        stats.last_set_stage_ms = ms;
        hcheck(hipEventElapsedTime(&ms, ev0, ev_mid));
        stats.last_encode_stage_ms = ms;
        hcheck(hipEventElapsedTime(&ms, ev_mid, ev1));
        stats.last_emit_kernel_ms = ms;
    }

    phase.mark("packed store + segment index");
    // ---- packed store + segment index
    // Every record the walk placed gets its bytes stored and its slot registered, even
    // if it failed later (emit / tokenize / the check above): later records of its
    // chunk may reference it, and the chunk's slot numbering must stay in step with
    // the device's.  A failed record is registered dead (not indexed).
    std::vector<uint8_t> placed(n);
    for (uint32_t r = 0; r < n; ++r)
        placed[r] = rchunk[r] != 0xffffffffu && ridx[r] != 0xffffffffu && doc_len[r] != 0xffffffffu &&
                    comp_len[r] <= 2 * doc_len[r] + 8;
    std::vector<uint64_t> coff(n + 1, 0), soff(n + 1, 0), loff(n + 1, 0), poff(n + 1, 0);
    std::vector<uint32_t> scap(n);
    const char *tsh = std::getenv("PX_DEBUG_TOKSEGS");
    const bool toksegs_check = tsh && tsh[0] == '1';
    if (n >= 65536) {  // (a million records: the four prefix sums on host threads)
        const uint32_t th = host_threads();
        parallel_ranges(n, th, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t r = lo; r < hi; ++r) {
                const bool ok = placed[r], parsed = !ok || (ntok[r] & kTokBad);
                scap[r] = (uint32_t)(parsed ? (ok ? seg_entries(nesc[r]) : 1)
                                            : std::min<uint64_t>(seg_entries(nesc[r]), 2ull * ntok[r] + 2));
            }
        });
        pxh::parallel_prefix(n, th, coff.data(), [&](uint32_t r) -> uint64_t { return placed[r] ? round_up(comp_len[r], 8) : 0; });
        pxh::parallel_prefix(n, th, soff.data(), [&](uint32_t r) -> uint64_t {
            const bool parsed = !placed[r] || (ntok[r] & kTokBad);
            return (parsed || toksegs_check ? scap[r] : 0) * sizeof(SegEnt);
        });
        pxh::parallel_prefix(n, th, loff.data(), [&](uint32_t r) -> uint64_t { return (uint64_t)scap[r] * sizeof(LaneEnt); });
        pxh::parallel_prefix(n, th, poff.data(),
                             [&](uint32_t r) -> uint64_t { return placed[r] ? round_up(pidx_blocks(doc_len[r]) * 2, 16) : 0; });
    } else
    for (uint32_t r = 0; r < n; ++r) {
        bool ok = placed[r];
        coff[r + 1] = coff[r] + (ok ? round_up(comp_len[r], 8) : 0);
        // room for the segment index: the encoder's tokens give it exactly (a plain segment
        // before each token, the tokens, the last plain bytes, the end sentinel); a record
        // whose tokens k_tok_segs cannot use is parsed by k_tokenize, which needs room for
        // every 251 of its bytes starting a token (seg_entries).  A failed record still gets
        // one entry: k_tokenize writes its end sentinel.  (Sizing every record by its 251
        // bytes gave config 4's records ~100 entries for the ~3 they use: 4.5 GB.)
        const bool parsed = !ok || (ntok[r] & kTokBad);
        const uint64_t ents = parsed ? (ok ? seg_entries(nesc[r]) : 1)
                                     : std::min<uint64_t>(seg_entries(nesc[r]), 2ull * ntok[r] + 2);
        scap[r] = (uint32_t)ents;
        // the lane entries hold everything a segment entry does for a record k_tok_segs
        // builds (16-bit source coordinates): such a record keeps no segment entries
        // (k_tokenize's records, whose coordinates may wrap, keep both)
        soff[r + 1] = soff[r] + (parsed || toksegs_check ? ents : 0) * sizeof(SegEnt);
        loff[r + 1] = loff[r] + ents * sizeof(LaneEnt);
        poff[r + 1] = poff[r] + (ok ? round_up(pidx_blocks(doc_len[r]) * 2, 16) : 0);
    }
    // compressed bytes and the lane entries share one allocation: a plain lane entry
    // reaches its record's bytes by a 32-bit relative offset (LaneEnt::rel)
    const uint64_t lane_at = round_up(coff[n] + 64, 16);
    const uint64_t store_bytes = lane_at + loff[n] + 64;
    auto *store = (uint8_t *)store_alloc(store_bytes);
    auto *segs = (uint8_t *)heap.alloc(soff[n] + poff[n] + 64);
    store_blocks.emplace_back(store, store_bytes);
    last_store = store;
    last_store_bytes = coff[n];
    store_blocks.emplace_back(segs, soff[n] + poff[n] + 64);
    macct.comp += lane_at;
    macct.lane += loff[n] + 64;
    macct.seg += soff[n];
    macct.pidx += poff[n] + 64;
    auto *d_coff = (uint64_t *)heap.alloc((uint64_t)n * 8);
    h2d(d_coff, coff.data(), (size_t)n * 8);
    hcheck(launch_compact(stream, n, d_cdst, d_complen, store, d_coff));
    // (the batch's slot entries in pinned memory kept across batches: copied to the device
    // straight from here, not through the bulk ring's staging copy -- 48 MB for a million records)
    auto *slots = static_cast<RecSlot *>(slot_pin.get((uint64_t)n * sizeof(RecSlot)));
    const uint32_t pthr = n >= 65536 ? host_threads() : 1;  // (per-record host loops of big batches)
    parallel_ranges(n, pthr, [&](uint32_t lo, uint32_t hi) {
    for (uint32_t r = lo; r < hi; ++r) {
        bool ok = placed[r];
        slots[r].comp = store + coff[r];
        slots[r].seg = soff[r + 1] > soff[r] ? (const SegEnt *)(segs + soff[r]) : nullptr;
        slots[r].pidx = (const uint16_t *)(segs + soff[n] + poff[r]);
        slots[r].comp_len = ok ? comp_len[r] : 0;
        slots[r].nseg = 0;
        slots[r].pidx_n = ok ? pidx_blocks(doc_len[r]) : 0;
        slots[r].seg_cap = scap[r];
        slots[r].lane = (const LaneEnt *)(store + lane_at + loff[r]);
    }
    });
    auto *d_slots = (RecSlot *)heap.alloc((uint64_t)n * sizeof(RecSlot));
    hcheck(hipMemcpyAsync(d_slots, slots, (size_t)n * sizeof(RecSlot), hipMemcpyHostToDevice, stream));
    std::vector<uint32_t> tstat(n);
    // segment index: from the encoder's tokens, then by parsing the bytes for the records that
    // could not be (k_tok_segs flags them)
    hcheck(launch_tok_segs(stream, n, d_slots, d_doclen, d_tokoff, d_toks, d_ntok, d_nseg, d_status));
    hcheck(launch_tokenize(stream, n, d_slots, d_nseg, d_status, d_ntok));
    std::vector<uint32_t> nseg(n);
    d2h(nseg.data(), d_nseg, n * 4);
    d2h(tstat.data(), d_status, n * 4);
    sync();
    if (toksegs_check) {  // test hook: the tokens' segment index == the bytes' parse
        const uint64_t seg_bytes = soff[n] + poff[n], lane_bytes = loff[n];
        std::vector<uint8_t> a(seg_bytes), al(lane_bytes), b(seg_bytes), bl(lane_bytes);
        std::vector<uint32_t> nseg2(n), tstat2(n);
        d2h(a.data(), segs, seg_bytes);
        d2h(al.data(), store + lane_at, lane_bytes);
        sync();
        hcheck(launch_tokenize(stream, n, d_slots, d_nseg, d_status, nullptr));
        d2h(b.data(), segs, seg_bytes);
        d2h(bl.data(), store + lane_at, lane_bytes);
        d2h(nseg2.data(), d_nseg, n * 4);
        d2h(tstat2.data(), d_status, n * 4);
        sync();
        uint32_t ntok_recs = 0;
        {
            std::vector<uint32_t> nt(n);
            d2h(nt.data(), d_ntok, n * 4);
            sync();
            for (uint32_t r = 0; r < n; ++r) ntok_recs += !(nt[r] & kTokBad);
        }
        for (uint32_t r = 0; r < n; ++r) {
            const uint64_t e = (nseg2[r] & ~(1u << 31)) + 1;  // entries incl. the sentinel
            const bool same = nseg[r] == nseg2[r] && tstat[r] == tstat2[r] &&
                              (!placed[r] || (std::memcmp(a.data() + soff[r], b.data() + soff[r], e * sizeof(SegEnt)) == 0 &&
                                              std::memcmp(al.data() + loff[r], bl.data() + loff[r], e * sizeof(LaneEnt)) == 0 &&
                                              std::memcmp(a.data() + soff[n] + poff[r], b.data() + soff[n] + poff[r],
                                                          pidx_blocks(doc_len[r]) * 2) == 0));
            if (!same) {
                fprintf(stderr, "pixiu_amd: record %u: segment index from tokens differs from the parse (nseg %u vs %u)\n", r,
                        nseg[r], nseg2[r]);
                throw PxFail{PX_ECORRUPT};
            }
        }
        fprintf(stderr, "pixiu_amd: segment index from tokens == parse for %u records (%u from tokens)\n", n, ntok_recs);
    }
    heap.release(d_toks, tok_n * sizeof(TokEnt) + 64);
    heap.release(d_tokoff, (uint64_t)n * 12 + 64);
    heap.release(comp_scratch, scratch_bytes + 256);
    heap.release(msgs, scratch_bytes * 4 + 256);
    heap.release(d_dst, (uint64_t)n * 8);
    heap.release(d_cdst, (uint64_t)n * 8);
    heap.release(d_coff, (uint64_t)n * 8);

    phase.mark("register records in their chunks");
    // ---- register records in their chunks
    std::vector<uint32_t> rgchunk(n, kNone);  // chunk of every placed record
    std::vector<uint8_t> live(n, 0);          // placed, OK and indexed
    // the chunks the batch opens, created in record order (global chunk ids as the serial
    // registration gave them); a chunk closed by a newer one gets its total once its records
    // are in.  Then every shard's records on host threads: a shard's chunks are its own.
    std::vector<uint32_t> closing;
    {
        // a shard's placed records go to nondecreasing chunks: each work's last chunk (its
        // records scanned on host threads for big batches), then the chunks opened in work order
        std::vector<int64_t> wmax(work.size(), -1);
        const std::function<void(uint32_t)> mx = [&](uint32_t k) {
            int64_t m = -1;
            for (uint32_t r = work[k].r0; r < work[k].r1; ++r)
                if (placed[r]) m = std::max<int64_t>(m, rchunk[r]);
            wmax[k] = m;
        };
        if (work.size() > 1 && n >= 65536) WorkerPool::get().run((uint32_t)work.size(), mx);
        else for (uint32_t k = 0; k < (uint32_t)work.size(); ++k) mx(k);
        for (size_t k = 0; k < work.size(); ++k) {
            Shard &s = *work[k].s;
            while (wmax[k] >= 0 && (int64_t)s.chunks.size() <= wmax[k]) {
                if (!s.chunks.empty()) closing.push_back(s.chunks.back());
                s.chunks.push_back(new_chunk(s.id));
            }
        }
    }
    struct RegAcc {
        uint64_t records = 0, raw = 0, doc = 0, comp = 0;
        int corrupt = 0;
    };
    std::vector<RegAcc> racc(work.size());
    auto register_work = [&](uint32_t k) {
        const Work &w = work[k];
        Shard &s = *w.s;
        RegAcc &a = racc[k];
        if (!s.chunks.empty()) {  // (the live chunk's tables grown once, not by doubling)
            Chunk &lc = chunks[s.chunks.back()];
            const size_t want = lc.n + (w.r1 - w.r0);
            auto grow = [want](auto &v) {  // (geometric: batches of one record stay amortised)
                if (v.capacity() < want) v.reserve(std::max(want, v.capacity() * 2));
            };
            grow(lc.slots);
            grow(lc.doc_len);
            grow(lc.dead);
            grow(lc.kp_off);
            grow(lc.kp_len);
        }
        for (uint32_t r = w.r0; r < w.r1; ++r) {
            if (doc_len[r] == 0xffffffffu) rstatus[r] = kErrInval;
            if (!placed[r]) continue;
            if (rstatus[r] == kOk && tstat[r] != kOk) rstatus[r] = tstat[r];
            uint32_t c = s.chunks[rchunk[r]];
            Chunk &ch = chunks[c];
            if (ridx[r] != ch.n) {  // the device numbered slots differently: fail loudly
                fprintf(stderr, "pixiu_amd: internal error: record %u placed at slot %u of chunk %u holding %u\n", r,
                        ridx[r], rchunk[r], ch.n);
                rstatus[r] = kErrCorrupt;
                a.corrupt = PX_ECORRUPT;
                continue;
            }
            const bool ok = rstatus[r] == kOk;
            set_nseg(slots[r], nseg[r]);
            ch.slots.push_back(slots[r]);
            ch.doc_len.push_back(doc_len[r]);
            ch.dead.push_back(ok ? 0 : 1);
            ch.kp_off.push_back(0);
            ch.kp_len.push_back(0);
            ch.n++;
            ch.used += ok ? 1 : 0;
            rgchunk[r] = c;
            live[r] = ok;
            if (!ok) continue;
            a.records++;
            a.raw += (hkoff[r + 1] - hkoff[r]) + (hvoff[r + 1] - hvoff[r]);
            a.doc += doc_len[r];
            a.comp += comp_len[r];
        }
    };
    if (work.size() > 1 && n >= 65536) {
        const std::function<void(uint32_t)> job = [&](uint32_t k) { register_work(k); };
        WorkerPool::get().run((uint32_t)work.size(), job);
    } else {
        for (uint32_t k = 0; k < (uint32_t)work.size(); ++k) register_work(k);
    }
    for (uint32_t c : closing) chunks[c].total = chunks[c].n;  // closed
    for (const RegAcc &a : racc) {
        stats.records += a.records;
        stats.raw_bytes += a.raw;
        stats.doc_bytes += a.doc;
        stats.comp_bytes += a.comp;
        if (a.corrupt) corrupt = a.corrupt;
    }
    phase.mark("register: slot tables and link jobs");
    // push new slot entries to the device tables and resolve the new records' tokens to
    // their target entries: per record its destination (the slots themselves are on the
    // device since k_tokenize), one kernel for both (k_slot_place), then k_link
    {
        std::vector<uint32_t> touched;
        {
            std::vector<uint8_t> seen(chunks.size(), 0);
            for (uint32_t r = 0; r < n; ++r)
                if (rgchunk[r] != kNone && !seen[rgchunk[r]]) {
                    seen[rgchunk[r]] = 1;
                    touched.push_back(rgchunk[r]);
                }
        }
        for (uint32_t c : touched) chunk_reserve(c, chunks[c].n);
        std::vector<SlotDst> sd(n);
        for (uint32_t r = 0; r < n; ++r) {
            if (rgchunk[r] == kNone) {
                sd[r] = SlotDst{nullptr, 0, 0};
                continue;
            }
            const Chunk &ch = chunks[rgchunk[r]];
            sd[r] = SlotDst{ch.dev + ridx[r], ridx[r], ch.n};
        }
        auto *d = (uint8_t *)slotput_buf.get(round_up((uint64_t)n * sizeof(SlotDst), 256) + (uint64_t)n * sizeof(LinkJob));
        auto *dsd = (SlotDst *)d;
        auto *dj = (LinkJob *)(d + round_up((uint64_t)n * sizeof(SlotDst), 256));
        h2d(dsd, sd.data(), (size_t)n * sizeof(SlotDst));
        hcheck(launch_slot_place(stream, n, d_slots, d_nseg, dsd, dj));
        hcheck(launch_link(stream, n, dj));
        sync();  // (d_slots and the job table are released / reused next)
        heap.release(d_slots, (uint64_t)n * sizeof(RecSlot));
    }

    phase.mark("compat key prefixes (GPU decode of each ");
    // ---- compat key prefixes (GPU decode of each new record's key region)
    {
        // the live records' jobs in record order (a prefix of the live flags places them, on host
        // threads for big batches)
        std::vector<uint64_t> lp(n + 1);
        const uint32_t th = n >= 65536 ? host_threads() : 1;
        pxh::parallel_prefix(n, th, lp.data(), [&](uint32_t r) -> uint64_t { return live[r] ? 1u : 0u; });
        std::vector<KpJob> jobs(lp[n]);
        std::vector<uint32_t> jrec(lp[n]);
        parallel_ranges(n, th, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t r = lo; r < hi; ++r) {
                if (!live[r]) continue;
                const uint64_t klen = hkoff[r + 1] - hkoff[r];
                // first decode's room: the key, its 251,0 and a few escapes (a prefix that does
                // not fit is decoded again with the whole doc's room; 1 M keys copied 2 klen + 66
                // bytes each down for ~klen + 2 used)
                jobs[lp[r]] = KpJob{rgchunk[r], ridx[r], doc_len[r], (uint32_t)std::min<uint64_t>(doc_len[r] + 64, klen + 2 + 30)};
                jrec[lp[r]] = r;
            }
        });
        std::vector<uint32_t> kst;
        decode_key_prefixes(jobs, kst);
        for (size_t i = 0; i < jobs.size(); ++i)
            if (kst[i] != kOk) {
                const uint32_t r = jrec[i];
                rstatus[r] = kst[i];
                chunks[rgchunk[r]].dead[ridx[r]] = 1;
                if (chunks[rgchunk[r]].used) chunks[rgchunk[r]].used--;
                live[r] = 0;
            }
    }

    phase.mark("device key index ids");
    // ---- device key index: ids for this batch's live records, in record order (before the
    // CritBit inserts, whose replaces kill ids -- older ones and this batch's own)
    const bool dk = dki_enabled() && dki.valid && !raw_docs;
    // ids are handed out here and written by dki_commit below: a batch that throws in
    // between leaves ids with no entry, so the index is then off until the next reset
    struct DkiTxn {
        px_ctx *c;
        bool done;
        ~DkiTxn() {
            if (!done) c->dki.valid = false;
        }
    } dk_txn{this, !dk};
    const uint32_t dk_gid0 = dki.nrec;
    // (the entries and key bytes are written into buffers kept across batches: value-
    // initialising a fresh 80 MB vector for a million records cost ~8 ms)
    DkRec *dk_new = nullptr;
    uint32_t dk_m = 0;
    std::vector<uint32_t> dk_r;  // the batch record of each entry
    std::vector<uint64_t> dk_kbo;  // its key bytes' place
    uint8_t *dk_kb = nullptr;
    uint64_t dk_kbn = 0;
    if (dk) {
        // live records in order: their ids and key-arena places by prefix sums, then the
        // entries on host threads (a batch of 1 M records spent ~45 ms here on one)
        {  // (the live records' list by a prefix of their flags, on host threads for big batches)
            std::vector<uint64_t> lp(n + 1);
            pxh::parallel_prefix(n, n >= 65536 ? host_threads() : 1, lp.data(), [&](uint32_t r) -> uint64_t { return live[r] ? 1u : 0u; });
            dk_r.resize(lp[n]);
            parallel_ranges(n, n >= 65536 ? host_threads() : 1, [&](uint32_t lo, uint32_t hi) {
                for (uint32_t r = lo; r < hi; ++r)
                    if (live[r]) dk_r[lp[r]] = r;
            });
        }
        const uint32_t m = (uint32_t)dk_r.size();
        std::vector<uint64_t> &kbo = dk_kbo;
        kbo.resize(m + 1);
        pxh::parallel_prefix(m, m >= 65536 ? host_threads() : 1, kbo.data(),
                             [&](uint32_t j) -> uint64_t { return hkoff[dk_r[j] + 1] - hkoff[dk_r[j]]; });
        {  // (every chunk's id table sized before the threads; new tables on host threads)
            std::vector<uint32_t> cs;
            for (const Work &w : work)
                for (uint32_t c : w.s->chunks)
                    if (chunks[c].gid.size() < chunks[c].n) cs.push_back(c);
            const std::function<void(uint32_t)> rs = [&](uint32_t i) { chunks[cs[i]].gid.resize(chunks[cs[i]].n, kNone); };
            if (cs.size() > 4 && n >= 65536) WorkerPool::get().run((uint32_t)cs.size(), rs);
            else for (uint32_t i = 0; i < (uint32_t)cs.size(); ++i) rs(i);
        }
        dk_new = static_cast<DkRec *>(dk_rec_pin.get((uint64_t)m * sizeof(DkRec) + 64));
        dk_m = m;
        dk_kb = static_cast<uint8_t *>(dk_key_pin.get(kbo[m] + 64));
        dk_kbn = kbo[m];
        const uint32_t gid0 = dki.nrec;
        dki.nrec += m;
        // ids now (the CritBit inserts below kill this batch's own replaced records by id)
        parallel_ranges(m, m >= 4096 ? host_threads() : 1, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t j = lo; j < hi; ++j) chunks[rgchunk[dk_r[j]]].gid[ridx[dk_r[j]]] = gid0 + j;
        });
    }

    phase.mark("span tables + CritBit inserts (concurrent)");
    // The CritBit inserts (host) run on a thread of their own while this one builds the span
    // tables (GPU decode, host sizing) and fills the index entries: neither reads what the
    // other writes (tries, dead marks and the key map there; span views and index entries
    // here), and their host-thread pool runs take turns.
    std::vector<uint32_t> replaced(n, 0);
    std::exception_ptr cb_err;
    std::thread cb_thread([&] {
        try {
    // ---- CritBit inserts: every shard's own records in arrival order, shards on host
    // threads (their tries are independent); then a key that moved to a newer shard is
    // deleted from its older one, in record order (a shard's records all precede a newer
    // shard's, so this is the order the sequential loop would have used)
    std::vector<std::pair<uint32_t, uint32_t>> moved;  // (record, older shard)
    // the key -> shard map's partitions (multi-shard stores) and the shards' tries are
    // independent: one pool run takes both (partitions first: the longer tasks)
    std::function<void(uint32_t)> keymap_job;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> mv;
    std::vector<std::string> rawk;
    if (opts.records_per_shard != 0) {
        // key -> shard upserts, one key-map partition per task (keys in record order); the
        // map holds raw keys: a ready doc's is its key prefix unescaped
        if (raw_docs) {
            rawk.resize(n);
            for (uint32_t r = 0; r < n; ++r) {
                if (!live[r]) continue;
                const uint8_t *d = hkeys.data() + hkoff[r];
                const uint32_t e = key_end(d, (uint32_t)(hkoff[r + 1] - hkoff[r]));
                std::string &k = rawk[r];
                for (uint32_t i = 0; i + 2 < e; ++i) {  // (e - 2: the 251,0 terminator)
                    k.push_back((char)d[i]);
                    if (d[i] == kEsc) ++i;  // 251,251 -> 251
                }
            }
        }
        auto raw_key = [&](uint32_t r, uint64_t *len) -> const uint8_t * {
            if (raw_docs) {
                *len = rawk[r].size();
                return reinterpret_cast<const uint8_t *>(rawk[r].data());
            }
            *len = hkoff[r + 1] - hkoff[r];
            return hkeys.data() + hkoff[r];
        };
        // every live key's hash (its partition is the top 4 bits), then each partition's
        // records in order as packed entries (hash, key, destination), so a task reads its
        // list sequentially and prefetches the slot and key bytes a few entries ahead (the
        // strided reads of per-record arrays, not the probes, were most of ~190 ns a key).
        // Both passes on host threads: per range of records, counts per partition, then the
        // entries scattered to (partition, range) offsets -- record order within a partition.
        constexpr uint32_t kRanges = 64;
        const uint32_t per = (n + kRanges - 1) / kRanges;
        std::vector<uint32_t> rcnt((size_t)kRanges * PartKeyMap::kParts, 0);
        khash.resize(n);
        const bool par = n >= 65536;
        const std::function<void(uint32_t)> count_job = [&](uint32_t t) {
            uint32_t *c = rcnt.data() + (size_t)t * PartKeyMap::kParts;
            for (uint32_t r = t * per, e = std::min(n, r + per); r < e; ++r)
                if (live[r]) {
                    uint64_t kl;
                    const uint8_t *kp = raw_key(r, &kl);
                    khash[r] = KeyMap::hash(kp, kl);
                    ++c[khash[r] >> 60];
                }
        };
        if (par) WorkerPool::get().run(kRanges, count_job);
        else for (uint32_t t = 0; t < kRanges; ++t) count_job(t);
        std::vector<uint64_t> roff((size_t)kRanges * PartKeyMap::kParts);  // (range, part) -> first entry
        uint64_t at = 0;
        for (uint32_t pi = 0; pi < PartKeyMap::kParts; ++pi) {
            pstart[pi] = at;
            for (uint32_t t = 0; t < kRanges; ++t) {
                roff[(size_t)t * PartKeyMap::kParts + pi] = at;
                at += rcnt[(size_t)t * PartKeyMap::kParts + pi];
            }
        }
        pstart[PartKeyMap::kParts] = at;
        if (kents.size() < at) kents.resize(at);
        const std::function<void(uint32_t)> fill_job = [&](uint32_t t) {
            uint64_t *o = roff.data() + (size_t)t * PartKeyMap::kParts;
            for (uint32_t r = t * per, e = std::min(n, r + per); r < e; ++r)
                if (live[r]) {
                    uint64_t kl;
                    const uint8_t *kp = raw_key(r, &kl);
                    kents[o[khash[r] >> 60]++] = KEnt{khash[r], kp, (uint32_t)kl, r, rec_shard[r], rgchunk[r], ridx[r]};
                }
        };
        if (par) WorkerPool::get().run(kRanges, fill_job);
        else for (uint32_t t = 0; t < kRanges; ++t) fill_job(t);
        mv.resize(PartKeyMap::kParts);
        keymap_job = [&](uint32_t pi) {
            KeyMap &m = keymap.part(pi);
            const KEnt *E = kents.data() + pstart[pi];
            const size_t ne = pstart[pi + 1] - pstart[pi];
            uint64_t kb = 0;
            for (size_t j = 0; j < ne; ++j) kb += E[j].klen;
            m.reserve(ne, kb);
            constexpr size_t kAhead = 8;
            for (size_t j = 0; j < ne; ++j) {
                if (j + kAhead < ne) {
                    __builtin_prefetch(m.probe_addr(E[j + kAhead].h));
                    __builtin_prefetch(E[j + kAhead].k);
                }
                const KEnt &e = E[j];
                const int64_t prev = m.upsert_h(e.h, e.k, e.klen, e.shard, e.chunk, e.idx);
                if (prev >= 0 && (uint32_t)prev != e.shard) mv[pi].emplace_back(e.r, (uint32_t)prev);
            }
        };
    }
    auto insert_work = [&](size_t k) {
        const Work &w = work[k];
        Shard &s = *w.s;
        std::string q;
        for (uint32_t r = w.r0; r < w.r1; ++r) {
            if (!live[r]) continue;
            if (raw_docs) {  // a ready doc: its escaped key is its prefix through 251,0
                const uint8_t *d = hkeys.data() + hkoff[r];
                q.assign(reinterpret_cast<const char *>(d), key_end(d, (uint32_t)(hkoff[r + 1] - hkoff[r])));
            } else {
                esc_key_into(q, hkeys.data() + hkoff[r], hkoff[r + 1] - hkoff[r]);
            }
            replaced[r] |= cbt_insert(s, q, Leaf{rgchunk[r], ridx[r]}) == 1 ? 1u : 0u;
        }
    };
    const uint32_t nk = keymap_job ? PartKeyMap::kParts : 0u;
    const uint32_t nthr = std::min<uint32_t>(host_threads(), (uint32_t)work.size() + nk);
    // (PX_SET_VERBOSE: every task's time, to see which kind sets the phase's length)
    std::vector<float> task_ms(phase.on ? nk + work.size() : 0);
    const std::function<void(uint32_t)> job = [&](uint32_t t) {
        const auto t0 = std::chrono::steady_clock::now();
        if (t < nk) keymap_job(t);
        else insert_work(t - nk);
        if (phase.on) task_ms[t] = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    if (nthr <= 1 || n < 2048) {
        for (uint32_t t = 0; t < nk + (uint32_t)work.size(); ++t) job(t);
    } else {
        // threads of its own, not the shared pool: the span build on the calling thread takes
        // the pool meanwhile (queued behind these tasks it waited ~6 ms for its first loop)
        static const uint32_t own = [] {
            const char *e = std::getenv("PX_CBT_THREADS");  // (0: the shared pool)
            return e ? (uint32_t)std::atoi(e) : 12u;  // (8: config 4's phase 18.5 ms; 12 / 16: 14.8 / 14.6, r06o)
        }();
        const uint32_t nt = std::min<uint32_t>(own, nk + (uint32_t)work.size());
        if (nt >= 2) {
            std::atomic<uint32_t> next{0};
            std::atomic<bool> stop{false};
            auto run = [&] {
                for (uint32_t t; !stop.load() && (t = next.fetch_add(1)) < nk + (uint32_t)work.size();) job(t);
            };
            std::vector<std::thread> th;
            th.reserve(nt - 1);
            std::exception_ptr err;
            std::mutex err_mu;
            auto guarded = [&] {
                try {
                    run();
                } catch (...) {
                    std::lock_guard<std::mutex> g(err_mu);
                    if (!err) err = std::current_exception();
                    stop.store(true);  // (the others stop taking tasks)
                }
            };
            for (uint32_t i = 1; i < nt; ++i) th.emplace_back(guarded);
            guarded();
            for (auto &x : th) x.join();
            if (err) std::rethrow_exception(err);
        } else {
            WorkerPool::get().run(nk + (uint32_t)work.size(), job);
        }
    }
    if (phase.on) {
        float km = 0, ks = 0, im = 0, is = 0;
        for (uint32_t t = 0; t < nk; ++t) km = std::max(km, task_ms[t]), ks += task_ms[t];
        for (uint32_t t = nk; t < task_ms.size(); ++t) im = std::max(im, task_ms[t]), is += task_ms[t];
        fprintf(stderr, "set_batch: key map tasks %u (max %.2f ms, sum %.2f), trie tasks %zu (max %.2f ms, sum %.2f), %u threads\n",
                nk, km, ks, work.size(), im, is, nthr);
    }
    for (auto &v : mv) moved.insert(moved.end(), v.begin(), v.end());
    std::sort(moved.begin(), moved.end());  // record order
    for (const auto &mv : moved) {  // cross-shard replace
        const uint32_t r = mv.first;
        cbt_delete(*shards[mv.second], crit_key(hkeys.data() + hkoff[r], hkoff[r + 1] - hkoff[r]));
        replaced[r] = 1;
    }

        } catch (...) {
            cb_err = std::current_exception();
        }
    });
    struct JoinGuard {  // (a throw on this thread still joins the inserts before unwinding)
        std::thread &t;
        ~JoinGuard() {
            if (t.joinable()) t.join();
        }
    } cb_guard{cb_thread};
    phase.mark("span tables of the new records (full-ran");
    // ---- span tables of the new records (full-range getitem as a gather)
    {
        std::vector<SpanReq> reqs;
        reqs.reserve(n);
        for (uint32_t r = 0; r < n; ++r)
            if (live[r]) reqs.push_back(SpanReq{rgchunk[r], ridx[r], dst[r]});
        const auto ts = std::chrono::steady_clock::now();
        build_spans(reqs);
        stats.last_span_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts).count();
    }

    if (dk) {  // the entries (span views, key bytes, clean flags) once the span tables exist
        const uint32_t m = dk_m;
        std::atomic<uint32_t> dk_max_len{0};
        parallel_ranges(m, m >= 4096 ? host_threads() : 1, [&](uint32_t lo, uint32_t hi) {
        std::string q;
        uint32_t lmax = 0;
        for (uint32_t j = lo; j < hi; ++j) {
            const uint32_t r = dk_r[j];
            Chunk &ch = chunks[rgchunk[r]];
            const uint32_t i = ridx[r];
            const uint8_t *k = hkeys.data() + hkoff[r];
            const uint64_t kl = hkoff[r + 1] - hkoff[r];
            DkRec d{};
            d.key_off = dki.keys_len + dk_kbo[j];
            d.key_len = (uint32_t)kl;
            if (kl) std::memcpy(dk_kb + dk_kbo[j], k, kl);
            if (i < ch.span.size() && ch.span[i].p) {
                const Chunk::Span &sp = ch.span[i];
                d.sp = sp.p;
                d.t = sp.t;
                d.n = sp.n;
                d.len = sp.len;
                if (sp.eq) {
                    d.xsp = sp.p;
                    d.xt = sp.t;
                    d.xn = sp.n;
                    d.xlen = sp.len;
                } else {
                    d.xsp = sp.xp;
                    d.xt = sp.xt;
                    d.xn = sp.xn;
                    d.xlen = sp.xlen;
                }
            }
            d.comp = ch.slots[i].comp;
            d.doc_len = ch.doc_len[i];
            esc_key_into(q, k, kl);
            const bool clean = kp_matches(Leaf{rgchunk[r], i}, q);
            d.flags = kDkLive | (clean ? kDkClean : 0u);  // (and in its trie: settled after the inserts)
            dk_new[j] = d;
            lmax = std::max({lmax, (uint32_t)d.len, (uint32_t)d.xlen});
        }
        uint32_t cur = dk_max_len.load();
        while (lmax > cur && !dk_max_len.compare_exchange_weak(cur, lmax)) {
        }
        });
        dki.max_len = std::max(dki.max_len, dk_max_len.load());
    }

    cb_thread.join();
    if (cb_err) std::rethrow_exception(cb_err);

    phase.mark("device key index");
    // a record the reference's CritBit skipped is answered by no walk: not by the index
    // either; a shard whose trie took an unclean prefix walks every lookup from now on
    for (uint32_t j = 0; j < dk_m; ++j)
        if (!chunks[rgchunk[dk_r[j]]].in_tree(ridx[dk_r[j]])) dk_new[j].flags &= ~kDkClean;
    for (const Work &w : work)
        if (w.s->unclean) dki.valid = false;
    if (dki.valid && dki_enabled()) {
        if (dk) dki_commit(dk_gid0, dk_new, dk_m, dk_kb, dk_kbn);
        dki_apply_kills();
    } else if (dki.nrec) {
        dki_clear();
    }
    dk_txn.done = true;

    for (auto &b : deferred_release) heap.release(b.first, b.second);
    deferred_release.clear();

    phase.mark("wait for the device");
    // ---- results (the batch's device work is done when the call returns: slot scatters
    // and span builds are not left running into the caller's next call)
    hcheck(hipStreamSynchronize(stream));
    phase.mark("results");
    int rc = corrupt;
    uint64_t ub = 0;
    for (auto &sp : shards) ub += sp->hs.ub_reads;
    stats.ub_reads = ub;
    stats.last_set_peak_bytes = heap.live_peak() + arena.mapped;
    trim_heap();
    stats.device_bytes = heap.held() + arena.mapped;
    for (uint32_t r = 0; r < n && rc == PX_OK; ++r) rc = map_status(rstatus[r]);
    if (res)
        parallel_ranges(n, n >= 65536 ? host_threads() : 1, [&](uint32_t lo, uint32_t hi) {
            for (uint32_t r = lo; r < hi; ++r) {
                const px_status st = map_status(rstatus[r]);
                px_set_result &o = res[r];
                o.status = st;
                o.replaced = replaced[r];
                o.shard = rec_shard[r];
                o.chunk = rchunk[r];
                o.idx = ridx[r];
                o.comp_len = st == PX_OK ? comp_len[r] : 0;
                o.doc_len = doc_len[r] == 0xffffffffu ? 0 : doc_len[r];
                o.pad = 0;
            }
        });
    return rc;
}

int px_ctx::expand(const std::vector<DecodeQuery> &q0, uint8_t *out, uint64_t out_cap, int out_on_device,
                   uint64_t *out_off, uint32_t *out_len, uint32_t *status, uint64_t *needed,
                   const std::vector<uint32_t> &pre_status) {
    const uint32_t n = (uint32_t)q0.size();
    std::vector<DecodeQuery> q = q0;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        out_off[i] = total;
        q[i].out_off = total;
        if (q[i].chunk != kNone) total += q[i].out_cap;
    }
    if (needed) *needed = total;
    if (total > out_cap) return PX_ESPACE;
    uint8_t *dout = out;
    if (!out_on_device) dout = (uint8_t *)in_buf.get(total + 64);
    std::vector<uint32_t> len, st;
    run_decode(q, dout, len, st, true);
    // queries that overran their slot: re-run with the exact size they need
    bool retry = false;
    for (uint32_t i = 0; i < n; ++i)
        if (q[i].chunk != kNone && st[i] == kErrSpace && q[i].out_cap < (uint32_t)kMaxDoc * 4) retry = true;
    if (retry) {
        // second pass with 4x room for the overflowing ones (over-yield is bounded)
        uint64_t t2 = 0;
        for (uint32_t i = 0; i < n; ++i) {
            if (q[i].chunk != kNone && st[i] == kErrSpace) q[i].out_cap = std::max<uint32_t>(q[i].out_cap * 4, 1024);
            out_off[i] = t2;
            q[i].out_off = t2;
            if (q[i].chunk != kNone) t2 += q[i].out_cap;
        }
        if (needed) *needed = t2;
        if (t2 > out_cap) return PX_ESPACE;
        if (!out_on_device) dout = (uint8_t *)in_buf.get(t2 + 64);
        run_decode(q, dout, len, st, true);
        total = t2;
    }
    int rc = PX_OK;
    for (uint32_t i = 0; i < n; ++i) {
        if (q[i].chunk == kNone) {
            out_len[i] = 0;
            status[i] = pre_status[i];
            continue;
        }
        out_len[i] = len[i];
        status[i] = map_status(st[i]);
        if (status[i] != PX_OK && rc == PX_OK) rc = (int)status[i];
    }
    if (!out_on_device) {
        d2h(out, dout, total);
        sync();
    }
    return rc;
}

// ====================================================================== reinsert
// PiXiuCtrl::setitem / delitem with the reinsert compaction (PiXiuCtrl.cpp:12-29, 63-69,
// 88-114).  A chunk closed with fewer than half of its records live is re-inserted: every
// live record, decoded through PXSGen (compat), goes back in through setitem as a ready
// doc and the CritBit replace deletes the old copy.  Triggers: the rotation that closes a
// chunk, and before every setitem / delitem the shard's Glob_Reinsert_Chunk (the last
// chunk a delete left under 80 % live).  The reference's loop visits all 65,535 slots and
// asserts each is set (PiXiuStr.cpp:189-193), so only slot-full chunks are defined; a
// chunk closed by the pool rule is left alone here (the reference dereferences NULL).
// Slot-full chunks exist only when a shard's live chunk can reach 65,535 records:
// records_per_shard = 0 (the reference's single instance).

namespace {
bool need_reinsert(const Chunk &c) { return c.total && c.used < 0.5 * c.total; }
}  // namespace

void px_ctx::reinsert_triggers(Shard &s, int when) {
    if (s.chunks.empty()) return;
    const uint32_t live = s.chunks.back();
    // the live chunk is slot-full: the next setitem rotates it (PiXiuCtrl.cpp:13-25).  The
    // rotation itself happens at the next doc the encoder places, so `closed` remembers
    // that this chunk's rotation trigger already ran (the reinsert below goes through
    // setitem again and would otherwise see the same full chunk).
    const bool rotating = s.hs.n_docs == (uint32_t)kChunkSlots;
    if (rotating && when != kTrigDel && s.closed != (int64_t)live) {
        s.closed = live;
        Chunk &ch = chunks[live];
        ch.total = ch.n;
        if (need_reinsert(ch)) {
            if (s.glob == (int64_t)live) s.glob = -1;
            reinsert_chunk(s, live, false);
        }
    }
    if (when == kTrigReinsert) return;
    // Glob_Reinsert_Chunk != st.cbt_chunk: delitem compares with the live chunk, setitem
    // with the chunk its record goes to (a new one when the live chunk is full)
    const int64_t cur = rotating && when == kTrigSet ? -2 : (int64_t)live;
    if (s.glob >= 0 && s.glob != cur && need_reinsert(chunks[(size_t)s.glob]))
        reinsert_chunk(s, (uint32_t)s.glob, true);
}

void px_ctx::reinsert_chunk(Shard &s, uint32_t c, bool via_glob) {
    if (chunks[c].n != (uint32_t)kChunkSlots) return;
    const int64_t curr = s.glob;
    // every live record, PXSGen-decoded over [0, 65535) (PiXiuCtrl.cpp:94-101)
    std::vector<DecodeQuery> q;
    uint64_t qo = 0;
    for (uint32_t i = 0; i < chunks[c].n; ++i) {
        if (chunks[c].dead[i]) continue;
        const uint32_t cap = (uint32_t)round_up(chunks[c].doc_len[i] + 64, 16);
        q.push_back(DecodeQuery{c, i, 0, kMaxDoc, qo, cap, 0});
        qo += cap;
    }
    std::vector<uint8_t> docs;
    std::vector<uint64_t> doff(1, 0);
    if (!q.empty()) {
        auto *dbuf = (uint8_t *)heap.alloc(qo + 64);
        std::vector<uint32_t> len, st;
        run_decode(q, dbuf, len, st, false);
        std::vector<uint8_t> h(qo);
        d2h(h.data(), dbuf, qo);
        sync();
        heap.release(dbuf, qo + 64);
        // a compat expansion longer than the doc (PXSGen's bug-compatible output) is
        // redone with the whole PXSG_MAX_TO window
        std::vector<DecodeQuery> q2;
        std::vector<uint32_t> which;
        uint64_t qo2 = 0;
        for (size_t k = 0; k < q.size(); ++k)
            if (st[k] == kErrSpace) {
                DecodeQuery d = q[k];
                d.out_off = qo2;
                d.out_cap = (uint32_t)round_up(kMaxDoc + 64, 16);
                qo2 += d.out_cap;
                q2.push_back(d);
                which.push_back((uint32_t)k);
            }
        std::vector<uint8_t> h2;
        std::vector<uint32_t> len2, st2;
        if (!q2.empty()) {
            auto *dbuf2 = (uint8_t *)heap.alloc(qo2 + 64);
            run_decode(q2, dbuf2, len2, st2, false);
            h2.resize(qo2);
            d2h(h2.data(), dbuf2, qo2);
            sync();
            heap.release(dbuf2, qo2 + 64);
        }
        for (size_t k = 0, j = 0; k < q.size(); ++k) {
            const uint8_t *src = h.data() + q[k].out_off;
            uint32_t l = len[k], stk = st[k];
            if (j < which.size() && which[j] == k) {
                src = h2.data() + q2[j].out_off;
                l = len2[j];
                stk = st2[j];
                ++j;
            }
            if (stk != kOk) throw PxFail{(int)map_status(stk)};
            l = std::min<uint32_t>(l, (uint32_t)kMaxDoc);  // the reference's uint16_t len
            docs.insert(docs.end(), src, src + l);
            doff.push_back(docs.size());
        }
    }
    // setitem(doc, reinsert = true) each, in slot order: rotation triggers only
    const bool saved = raw_docs;
    raw_docs = true;
    const uint32_t n = (uint32_t)q.size();
    std::vector<uint64_t> zero(n + 1, 0);
    uint8_t dummy = 0;
    for (uint32_t pos = 0; pos < n;) {
        reinsert_triggers(s, kTrigReinsert);
        const uint32_t room = (uint32_t)kChunkSlots - std::min<uint32_t>(s.hs.n_docs, kChunkSlots);
        const uint32_t end = std::min(n, pos + std::max(room, 1u));
        std::vector<uint64_t> off(doff.begin() + pos, doff.begin() + end + 1);
        const int rc = set_batch(end - pos, docs.data(), off.data(), &dummy, zero.data(), 0, nullptr);
        if (rc != PX_OK) {
            raw_docs = saved;
            throw PxFail{rc};
        }
        pos = end;
    }
    raw_docs = saved;
    // PiXiuChunk_free: the chunk's records are gone (and out of the device key index: a record
    // whose re-set CritBit insert was skipped would otherwise still be answered from here)
    Chunk &ch = chunks[c];
    for (uint32_t i = 0; i < ch.n && i < ch.gid.size(); ++i)
        if (!ch.dead[i] && ch.gid[i] != kNone) dki.kills.push_back(ch.gid[i]);
    std::fill(ch.dead.begin(), ch.dead.end(), (uint8_t)1);
    ch.used = 0;
    s.glob = via_glob ? -1 : curr;
}

int px_ctx::set_ctrl(uint32_t n, const uint8_t *keys, const uint64_t *koff, const uint8_t *vals,
                     const uint64_t *voff, int on_device, px_set_result *res) {
    if (opts.records_per_shard != 0 || n == 0) return set_batch(n, keys, koff, vals, voff, on_device, res);
    // one shard (the reference's single instance): evaluate the triggers between records
    std::vector<uint64_t> ko(n + 1), vo(n + 1);
    std::vector<uint8_t> hk, hv;
    if (on_device) {
        d2h(ko.data(), koff, (size_t)(n + 1) * 8);
        d2h(vo.data(), voff, (size_t)(n + 1) * 8);
        sync();
    } else {
        std::memcpy(ko.data(), koff, (size_t)(n + 1) * 8);
        std::memcpy(vo.data(), voff, (size_t)(n + 1) * 8);
    }
    Shard *s = shards.empty() ? nullptr : shards[0].get();
    bool full_closed = false;  // a slot-full closed chunk exists: a replace may move Glob onto it
    if (s)
        for (uint32_t c : s->chunks) full_closed |= chunks[c].total == (uint32_t)kChunkSlots;
    const bool fast = !s || (s->hs.n_docs + (uint64_t)n < (uint64_t)kChunkSlots && !full_closed);
    if (fast) return set_batch(n, keys, koff, vals, voff, on_device, res);
    if (on_device) {  // the slow path reads keys on the host
        hk.resize(ko[n] - ko[0]);
        hv.resize(vo[n] - vo[0]);
        d2h(hk.data(), keys + ko[0], hk.size());
        d2h(hv.data(), vals + vo[0], hv.size());
        sync();
        const uint64_t k0 = ko[0], v0 = vo[0];
        for (auto &o : ko) o -= k0;
        for (auto &o : vo) o -= v0;
        keys = hk.data();
        vals = hv.data();
        on_device = 0;
    }
    int rc = PX_OK;
    for (uint32_t pos = 0; pos < n;) {
        s = shards.empty() ? nullptr : shards[0].get();
        uint32_t end = n;
        if (s) {
            reinsert_triggers(*s, kTrigSet);
            const uint32_t room = (uint32_t)kChunkSlots - std::min<uint32_t>(s->hs.n_docs, kChunkSlots);
            end = std::min(n, pos + std::max(room, 1u));
            full_closed = false;
            for (uint32_t c : s->chunks) full_closed |= chunks[c].total == (uint32_t)kChunkSlots;
            if (full_closed) {
                // stop after the first record whose replace leaves a slot-full closed chunk
                // under half live: Glob then triggers before the next record
                std::unordered_map<uint32_t, uint32_t> dec;
                std::unordered_set<std::string> seen;
                for (uint32_t r = pos; r < end; ++r) {
                    std::string q = crit_key(keys + ko[r], ko[r + 1] - ko[r]);
                    Leaf l;
                    if (!seen.insert(q).second || !cbt_lookup(*s, q, &l)) continue;
                    const Chunk &ch = chunks[l.chunk];
                    if (ch.total != (uint32_t)kChunkSlots || ch.dead[l.idx]) continue;
                    const uint32_t d = ++dec[l.chunk];
                    if (ch.used - std::min(d, ch.used) < 0.5 * ch.total) {
                        end = r + 1;
                        break;
                    }
                }
            }
        }
        const int r2 = set_batch(end - pos, keys, ko.data() + pos, vals, vo.data() + pos, on_device,
                                 res ? res + pos : nullptr);
        if (rc == PX_OK) rc = r2;
        pos = end;
    }
    return rc;
}

// Write-behind setitem (px_opts.defer_bytes; include/pixiu_amd.h px_flush).  `replaced`
// (CBT_SET_REPLACE, CritBitTree.cpp:32-43) is resolved at call time: the key is in the
// CritBit of the stored records (the same lookup contains() makes) or equals a queued
// key -- and a key equal to a queued one flushes the queue first, so the earlier record
// is stored and the lookup exact.  The one case this cannot see is a queued record
// whose compat-decoded key (what the reference's CritBit compares, CritBitTree.cpp:27-28)
// is not its key, i.e. the reference decoder's bug inside a key; flush_queue counts any
// such difference in stats.deferred_mismatch and says so on stderr.
int px_ctx::set_deferred(uint32_t n, const uint8_t *keys, const uint64_t *koff, const uint8_t *vals,
                         const uint64_t *voff, px_set_result *res) {
    std::string q;
    int rc = PX_OK;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t *k = keys + koff[i];
        const uint64_t kn = koff[i + 1] - koff[i], vn = voff[i + 1] - voff[i];
        const uint8_t *v = vn ? vals + voff[i] : nullptr;
        uint64_t esc = 0;
        for (uint64_t j = 0; j < kn; ++j) esc += k[j] == kEsc;
        for (uint64_t j = 0; j < vn; ++j) esc += v[j] == kEsc;
        const uint64_t dl = kn + 2 + (vn ? vn + 2 : 0) + esc;  // PiXiuCtrl.cpp:31-44
        px_set_result r{PX_OK, 0, 0, PX_PENDING, PX_PENDING, PX_PENDING, (uint32_t)dl, 0};
        if (kn == 0 || dl > (uint64_t)kMaxDoc) {  // as k_doc_len: never placed
            r = px_set_result{PX_EINVAL, 0, 0, 0xffffffffu, 0xffffffffu, 0, 0, 0};
            if (rc == PX_OK) rc = PX_EINVAL;
            if (res) res[i] = r;
            continue;
        }
        esc_key_into(q, k, kn);
        if (dq_keys.count(q)) flush_queue();
        Shard *s = shards.empty() ? nullptr : shards[0].get();
        r.replaced = (dq_keys.count(q) || (s && cbt_contains(*s, q))) ? 1u : 0u;
        dq_k.insert(dq_k.end(), k, k + kn);
        if (vn) dq_v.insert(dq_v.end(), v, v + vn);
        dq_ko.push_back(dq_k.size());
        dq_vo.push_back(dq_v.size());
        dq_pred.push_back(r.replaced);
        dq_keys.insert(q);
        stats.deferred_records++;
        if (res) res[i] = r;
        if (dq_k.size() + dq_v.size() >= opts.defer_bytes || dq_pred.size() >= (size_t)kChunkSlots) flush_queue();
    }
    return rc;
}

int px_ctx::flush_queue() {
    const uint32_t n = (uint32_t)dq_pred.size();
    if (!n) return PX_OK;
    std::vector<px_set_result> r(n);
    uint8_t dummy = 0;
    // (moved out first: set_ctrl's reinsert triggers may re-enter nothing here, and a
    // failure below must not leave the records queued twice)
    std::vector<uint8_t> k, v;
    std::vector<uint64_t> ko, vo;
    std::vector<uint32_t> pred;
    k.swap(dq_k);
    v.swap(dq_v);
    ko.swap(dq_ko);
    vo.swap(dq_vo);
    pred.swap(dq_pred);
    drop_queue();
    stats.deferred_flushes++;
    int rc;
    try {
        rc = set_ctrl(n, k.data(), ko.data(), v.empty() ? &dummy : v.data(), vo.data(), 0, r.data());
    } catch (...) {
        // the queued records are gone with the failed batch: the caller that triggered the
        // flush gets the error from PX_GUARD, and px_flush reports it afterwards too
        int code = PX_EHIP;
        try {
            throw;
        } catch (const PxFail &f) {
            code = f.code;
        } catch (const std::bad_alloc &) {
            code = PX_ENOMEM;
        } catch (...) {
        }
        if (dq_rc == PX_OK) dq_rc = code;
        throw;
    }
    uint64_t mism = 0;
    for (uint32_t i = 0; i < n; ++i) mism += r[i].status == PX_OK && r[i].replaced != pred[i];
    if (mism) {
        stats.deferred_mismatch += mism;
        fprintf(stderr, "pixiu_amd: %llu deferred setitem result(s) returned replaced != the stored result "
                        "(a queued record's compat-decoded key differs from its key)\n", (unsigned long long)mism);
    }
    note_last(n, r.data());
    if (rc != PX_OK && dq_rc == PX_OK) dq_rc = rc;
    return rc;
}

// ====================================================================== device key index
void px_ctx::dki_commit(uint32_t gid0, const DkRec *recs, uint32_t nn, const uint8_t *kb, uint64_t kbn) {
    if (!nn) return;
    dki.miss_streak = 0;
    if (!dki.err) {
        dki.err = (uint32_t *)heap.alloc(256);
        hcheck(hipMemsetAsync(dki.err, 0, 256, stream));
    }
    const uint64_t need_rec = (uint64_t)gid0 + nn;
    if (need_rec > dki.rec_cap) {  // (records only grow; ids are positions in this array)
        const uint64_t cap = std::max<uint64_t>(need_rec, std::max<uint64_t>(4096, dki.rec_cap * 2));
        auto *nr = (DkRec *)heap.alloc(cap * sizeof(DkRec));
        if (dki.rec) {
            hcheck(hipMemcpyAsync(nr, dki.rec, (size_t)gid0 * sizeof(DkRec), hipMemcpyDeviceToDevice, stream));
            deferred_release.emplace_back(dki.rec, dki.rec_cap * sizeof(DkRec));
        }
        dki.rec = nr;
        dki.rec_cap = cap;
    }
    if (dki.keys_len + kbn + 16 > dki.keys_cap) {  // (16 bytes of slack: the index reads 16 at a time)
        const uint64_t cap =
            std::max<uint64_t>(dki.keys_len + kbn + 16, std::max<uint64_t>(1 << 16, dki.keys_cap * 2));
        auto *nk = (uint8_t *)heap.alloc(cap);
        if (dki.keys) {
            hcheck(hipMemcpyAsync(nk, dki.keys, dki.keys_len, hipMemcpyDeviceToDevice, stream));
            deferred_release.emplace_back(dki.keys, dki.keys_cap);
        }
        dki.keys = nk;
        dki.keys_cap = cap;
    }
    // (recs / kb are pinned and stay untouched until the batch's closing stream sync)
    hcheck(hipMemcpyAsync(dki.rec + gid0, recs, (size_t)nn * sizeof(DkRec), hipMemcpyHostToDevice, stream));
    if (kbn) hcheck(hipMemcpyAsync(dki.keys + dki.keys_len, kb, kbn, hipMemcpyHostToDevice, stream));
    dki.keys_len += kbn;
    uint32_t first = gid0, count = nn;
    if ((uint64_t)dki.nrec * 2 > dki.tab_cap) {  // a new table: every record again (newest id wins)
        uint32_t cap = 1024;
        while ((uint64_t)cap < (uint64_t)dki.nrec * 2) cap <<= 1;
        if (dki.tab) deferred_release.emplace_back(dki.tab, (uint64_t)dki.tab_cap * sizeof(DkSlot));
        dki.tab = (DkSlot *)heap.alloc((uint64_t)cap * sizeof(DkSlot));
        dki.tab_cap = cap;
        hcheck(hipMemsetAsync(dki.tab, 0, (size_t)cap * sizeof(DkSlot), stream));
        first = 0;
        count = dki.nrec;
    }
    hcheck(launch_dk_insert(stream, first, count, dki.rec, dki.keys, dki.tab, dki.tab_cap - 1, dki.err));
}

// getitem through the device key index into a device buffer.  Returns -1 (nothing
// written, nothing reported) when any key is not one the index answers, or the output
// does not fit: the caller then runs the host path, so results never depend on this.
int px_ctx::dki_get(uint32_t n, const uint8_t *keys, const uint64_t *koff, int mode, uint8_t *out, uint64_t out_cap,
                    int out_on_device, uint64_t *out_off, uint32_t *out_len, uint32_t *status, uint64_t *needed,
                    bool dev_io) {
    if (!dki_enabled() || !dki.valid || !dki.tab || !n || !spans_enabled()) return -1;
    // a store whose batches keep missing (8 in a row: records the index does not hold, e.g. reinserted or
    // set as ready docs) tries it only every 16th batch until a set batch adds records
    if (dki.miss_streak >= 8 && (++dki.skipped & 15)) return -1;
    PhaseClock phase("dki_get", "PX_GET_VERBOSE");
    phase.mark("kills, scratch, keys to pinned");
    dki_apply_kills();  // (deletes since the last set batch)
    const uint64_t k0 = dev_io ? 0 : koff[0], kbytes = dev_io ? 0 : koff[n] - k0;  // (device keys: read in place)
    // device scratch: keys, offsets, gather queries, the look-back chain, then what comes back
    // in one copy (ctl: misses, output / 16, tiles, insert error, ticket; offsets out; lengths;
    // statuses), then the gather's task table
    const uint64_t nb = (n + 255) / 256;
    const uint64_t o_off = round_up(kbytes + 16, 256), o_gq = o_off + round_up((uint64_t)(n + 1) * 8, 256),
                   o_chain = o_gq + round_up((uint64_t)n * sizeof(GatherQuery), 256), o_ctl = o_chain + nb * 16,
                   o_oo = o_ctl + 32, o_dl = o_oo + (uint64_t)n * 4, o_ds = o_dl + (uint64_t)n * 4,
                   o_end = o_ds + (uint64_t)n * 4, o_task = round_up(o_end, 256);
    // the tasks: at most one per 64 tiles, a tile per 16 bytes of the output that fits
    // (every query's tiles <= its cap / 16), so the launch can go before the totals are known
    // (a host buffer: device staging up to 4 GiB; a batch past it goes the host path)
    // (output offsets travel as u32 counts of 16 bytes: below 64 GiB on the device too)
    const uint64_t cap_fit = std::min<uint64_t>(out_cap, out_on_device ? (1ull << 36) - 16 : 4ull << 30);
    // (and by the index's longest expansion: a query's tiles are at most max(1, ceil(max_len /
    // 32)), 64 tiles a task -- a grid sized from the caller's room alone was 4x the batch's real
    // tasks on config 3, every spare wave dispatched only to exit)
    const uint64_t tiles_q = std::max<uint64_t>(1, ((uint64_t)dki.max_len + kGatherTile - 1) / kGatherTile);
    const uint64_t ntask_max =
        std::min<uint64_t>({cap_fit / 1024 + 2, (uint64_t)n * tiles_q / 64 + 2, 0xffffffffull});
    auto *b = (uint8_t *)dk_qbuf.get(o_task + gather_task_bytes((uint32_t)ntask_max));
    auto *dkeys = dev_io ? const_cast<uint8_t *>(keys) : b;
    auto *doff = dev_io ? const_cast<uint64_t *>(koff) : (uint64_t *)(b + o_off);
    auto *gq = (GatherQuery *)(b + o_gq);
    auto *chain = (unsigned long long *)(b + o_chain);
    auto *ctl = (uint32_t *)(b + o_ctl);
    auto *oo = (uint32_t *)(b + o_oo);  // output offsets in 16-byte units
    auto *dl = (uint32_t *)(b + o_dl), *ds = (uint32_t *)(b + o_ds);
    void *task = b + o_task;
    // keys up through pinned memory (one copy of the bytes and the rebased offsets)
    auto *hb = (uint8_t *)dk_hbuf.get(o_gq);
    auto *ho = (uint64_t *)(hb + o_off);
    // (a million-key batch: 16 MB staged on the host threads, in parts whose uploads start
    // while the next part is staged)
    const uint32_t parts = dev_io ? 0u : n >= 65536 ? 4u : 1u;
    for (uint32_t part = 0; part < parts; ++part) {
        const uint32_t r0 = (uint32_t)((uint64_t)(n + 1) * part / parts), r1 = (uint32_t)((uint64_t)(n + 1) * (part + 1) / parts);
        parallel_ranges(r1 - r0, n >= 65536 ? host_threads() : 1, [&](uint32_t lo, uint32_t hi) {
            lo += r0;
            hi += r0;
            const uint64_t a = koff[lo] - k0, b = (hi > n ? koff[n] : koff[hi]) - k0;
            std::memcpy(hb + a, keys + k0 + a, b - a);
            for (uint32_t i = lo; i < hi; ++i) ho[i] = koff[i] - k0;
        });
        // (part p uploads its key bytes and offsets; the last part also the bytes' tail to o_off)
        const uint64_t ka = koff[r0] - k0, kb = part + 1 == parts ? o_off : (r1 > n ? koff[n] : koff[r1]) - k0;
        hcheck(hipMemcpyAsync(dkeys + ka, hb + ka, kb - ka, hipMemcpyHostToDevice, stream));
        hcheck(hipMemcpyAsync(doff + r0, ho + r0, (uint64_t)(r1 - r0) * 8, hipMemcpyHostToDevice, stream));
    }
    phase.mark("launches");
    hcheck(hipMemsetAsync(chain, 0, nb * 16 + 32, stream));
    flush_tab();
    hcheck(hipEventRecord(ev0, stream));
    hcheck(launch_dk_lookup(stream, n, dkeys, doff, dki.tab, dki.tab_cap - 1, dki.rec, dki.keys, (uint32_t)mode, gq,
                            oo, ctl, chain, dki.err));
    // (a host output buffer: gathered into device staging of cap_fit bytes, then copied down)
    uint8_t *dout = out_on_device ? out : (uint8_t *)dk_obuf.get(cap_fit + 64);
    hcheck(launch_gather(stream, (uint32_t)ntask_max, ctl, cap_fit, task, gq, n, dout, dl, ds));
    hcheck(hipEventRecord(ev1, stream));
    // one copy, one round trip: ctl, offsets and lengths (the statuses only when some query
    // ran past its room, ctl[5]); device results: the results kernel, then ctl alone
    auto *hr = (uint32_t *)dk_hres.get(o_end - o_ctl);
    if (dev_io) hcheck(launch_dk_results(stream, n, ctl, cap_fit, oo, dl, ds, out_off, out_len, status));
    hcheck(hipMemcpyAsync(hr, ctl, dev_io ? 32 : o_ds - o_ctl, hipMemcpyDeviceToHost, stream));
    phase.mark("wait for the device");
    spin_sync();
    phase.mark("results");
    const uint8_t *res = (const uint8_t *)hr + 32;
    if (hr[3]) {  // an insert gave up: the index is not trusted again until reset
        fprintf(stderr, "pixiu_amd: device key index insert failed; getitem resolves on the host\n");
        dki.valid = false;
        return -1;
    }
    const uint64_t total = (uint64_t)hr[1] * 16;
    if (dev_io && !hr[0] && total > out_cap) {  // (device results: too little room is the caller's answer)
        if (needed) *needed = total;
        return PX_ESPACE;
    }
    if (hr[0] || total > cap_fit) {  // (nothing was gathered: the host path answers)
        dki.miss_streak += hr[0] ? 1 : 0;
        return -1;
    }
    dki.miss_streak = 0;
    if (!out_on_device && total) {
        d2h(out, dout, total);
        sync();  // (d2h may finish through pinned staging at the sync)
    }
    float ms = 0;
    hcheck(hipEventElapsedTime(&ms, ev0, ev1));
    stats.last_decode_kernel_ms = ms;
    stats.last_gather_queries = n;
    stats.last_get_device_keys = n;
    if (dev_io) {  // (the results kernel wrote offsets, lengths and statuses)
        if (needed) *needed = total;
        return hr[5] ? PX_ESPACE : PX_OK;
    }
    const uint32_t *ro = (const uint32_t *)res, *rl = ro + n;
    const uint32_t *rs = nullptr;
    if (hr[5]) {  // (statuses only when some query ran past its room)
        uint32_t *h = (uint32_t *)dk_hres.get(o_end - o_ctl) + (o_ds - o_ctl) / 4;
        hcheck(hipMemcpy(h, ds, (size_t)n * 4, hipMemcpyDeviceToHost));
        rs = h;
    }
    parallel_ranges(n, n >= 65536 ? host_threads() : 1, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i) out_off[i] = (uint64_t)ro[i] * 16;
        std::memcpy(out_len + lo, rl + lo, (size_t)(hi - lo) * 4);
        if (rs)
            for (uint32_t i = lo; i < hi; ++i) status[i] = map_status(rs[i]);
        else
            std::fill(status + lo, status + hi, (uint32_t)PX_OK);
    });
    int rc = PX_OK;
    if (rs)
        for (uint32_t i = 0; i < n; ++i)
            if (status[i] != PX_OK) {
                rc = (int)status[i];
                break;
            }
    if (needed) *needed = total;
    return rc;
}

int px_ctx::del_ctrl(uint32_t n, const uint8_t *keys, const uint64_t *koff, uint32_t *result) {
    for (uint32_t i = 0; i < n; ++i) {
        Shard *s = shard_for_key(keys + koff[i], koff[i + 1] - koff[i]);
        if (s && opts.records_per_shard == 0) reinsert_triggers(*s, kTrigDel);  // PiXiuCtrl.cpp:64-67
        result[i] = s ? (uint32_t)cbt_delete(*s, esc_key(keys + koff[i], koff[i + 1] - koff[i])) : 1u;
    }
    return PX_OK;
}

// ====================================================================== chunk blob
// Wire / on-disk format v1 of stored records (include/pixiu_amd.h px_save; SURVEY.md
// §8f row 3 -- the reference has no persistence).  Little-endian:
//   BlobHeader (64 B) | BlobChunk x n_chunks | BlobRec x n_records | data
// data holds every record's compressed bytes, each 8-byte aligned, in chunk order.
namespace {
constexpr uint32_t kBlobMagic = 0x42435850u;  // "PXCB"
constexpr uint32_t kBlobVersion = 1;
constexpr uint32_t kBlobDead = 1u << 31;  // BlobRec::doc_len flag: deleted / failed record
struct BlobHeader {
    uint32_t magic, version, n_chunks, n_records;
    uint64_t data_off, data_bytes;
    uint32_t flags, pad[7];
};
struct BlobChunk {
    uint32_t shard, seq, first, n;  // source shard, chunk sequence in it, first record, records
};
struct BlobRec {
    uint64_t off;  // into data
    uint32_t comp_len, doc_len;  // doc_len | kBlobDead
};
static_assert(sizeof(BlobHeader) == 64 && sizeof(BlobChunk) == 16 && sizeof(BlobRec) == 16, "blob layout");
}  // namespace

int px_ctx::save(uint8_t *dst, uint64_t cap, int dst_on_device, uint64_t *bytes) {
    std::vector<BlobChunk> bc;
    std::vector<BlobRec> br;
    std::vector<const uint8_t *> src;
    uint64_t data = 0;
    for (auto &sp : shards)
        for (uint32_t seq = 0; seq < sp->chunks.size(); ++seq) {
            const Chunk &ch = chunks[sp->chunks[seq]];
            if (!ch.n) continue;
            bc.push_back(BlobChunk{sp->id, seq, (uint32_t)br.size(), ch.n});
            for (uint32_t i = 0; i < ch.n; ++i) {
                const RecSlot &sl = ch.slots[i];
                br.push_back(BlobRec{data, sl.comp_len, ch.doc_len[i] | (ch.dead[i] ? kBlobDead : 0u)});
                src.push_back(sl.comp);
                data += round_up(sl.comp_len, 8);
            }
        }
    BlobHeader h{};
    h.magic = kBlobMagic;
    h.version = kBlobVersion;
    h.n_chunks = (uint32_t)bc.size();
    h.n_records = (uint32_t)br.size();
    h.data_off = round_up(sizeof(BlobHeader) + bc.size() * sizeof(BlobChunk) + br.size() * sizeof(BlobRec), 64);
    h.data_bytes = data;
    const uint64_t total = h.data_off + data;
    if (bytes) *bytes = total;
    if (!dst) return PX_OK;
    if (cap < total) return PX_ESPACE;
    std::vector<uint8_t> head(h.data_off, 0);
    std::memcpy(head.data(), &h, sizeof h);
    std::memcpy(head.data() + sizeof h, bc.data(), bc.size() * sizeof(BlobChunk));
    std::memcpy(head.data() + sizeof h + bc.size() * sizeof(BlobChunk), br.data(), br.size() * sizeof(BlobRec));
    // pack the records' bytes on the device (k_compact), then place the blob
    uint8_t *pack = dst_on_device ? dst : (uint8_t *)heap.alloc(total + 64);
    const uint32_t n = h.n_records;
    if (n) {
        auto *d_src = (uint8_t **)heap.alloc((uint64_t)n * 8);
        auto *d_len = (uint32_t *)heap.alloc((uint64_t)n * 4);
        auto *d_off = (uint64_t *)heap.alloc((uint64_t)n * 8);
        std::vector<uint32_t> len(n);
        std::vector<uint64_t> off(n);
        for (uint32_t i = 0; i < n; ++i) {
            len[i] = br[i].comp_len;
            off[i] = br[i].off;
        }
        h2d(d_src, src.data(), (size_t)n * 8);
        h2d(d_len, len.data(), (size_t)n * 4);
        h2d(d_off, off.data(), (size_t)n * 8);
        hcheck(hipMemsetAsync(pack + h.data_off, 0, data, stream));  // alignment padding is zero
        hcheck(launch_compact(stream, n, d_src, d_len, pack + h.data_off, d_off));
        sync();
        heap.release(d_src, (uint64_t)n * 8);
        heap.release(d_len, (uint64_t)n * 4);
        heap.release(d_off, (uint64_t)n * 8);
    }
    if (dst_on_device) {
        h2d(dst, head.data(), head.size());
        sync();
    } else {
        std::memcpy(dst, head.data(), head.size());
        d2h(dst + h.data_off, pack + h.data_off, data);
        sync();
        heap.release(pack, total + 64);
    }
    return PX_OK;
}

int px_ctx::load(const uint8_t *src, uint64_t len, int src_on_device, uint32_t *first_shard) {
    if (len < sizeof(BlobHeader)) return PX_EINVAL;
    BlobHeader h;
    if (src_on_device) {
        d2h(&h, src, sizeof h);
        sync();
    } else {
        std::memcpy(&h, src, sizeof h);
    }
    const uint64_t tables = sizeof(BlobHeader) + (uint64_t)h.n_chunks * sizeof(BlobChunk) +
                            (uint64_t)h.n_records * sizeof(BlobRec);
    if (h.magic != kBlobMagic || h.version != kBlobVersion || h.data_off < tables || h.data_off > len ||
        h.data_bytes > len - h.data_off)
        return PX_EINVAL;
    std::vector<uint8_t> tab(tables);
    if (src_on_device) {
        d2h(tab.data(), src, tables);
        sync();
    } else {
        std::memcpy(tab.data(), src, tables);
    }
    std::vector<BlobChunk> bc(h.n_chunks);
    std::vector<BlobRec> br(h.n_records);
    std::memcpy(bc.data(), tab.data() + sizeof h, bc.size() * sizeof(BlobChunk));
    std::memcpy(br.data(), tab.data() + sizeof h + bc.size() * sizeof(BlobChunk), br.size() * sizeof(BlobRec));
    // validate: chunks tile the records in order, each shard's chunks are 0..k-1
    uint64_t next = 0;
    std::map<uint32_t, uint32_t> seqs;  // source shard -> chunks seen
    for (const BlobChunk &c : bc) {
        if (c.first != next || c.n == 0 || c.n > (uint32_t)kChunkSlots || c.seq != seqs[c.shard]) return PX_EINVAL;
        seqs[c.shard]++;
        next += c.n;
    }
    if (next != h.n_records) return PX_EINVAL;
    for (const BlobRec &r : br)
        if ((r.doc_len & ~kBlobDead) > (uint32_t)kMaxDoc || r.comp_len > (uint32_t)kMaxDoc ||
            r.off + r.comp_len > h.data_bytes || (r.off & 7))
            return PX_EINVAL;
    // single-shard stores take the blob's chunks into shard 0, which must be empty
    if (opts.records_per_shard == 0 && !shards.empty() && shards[0]->records) return PX_EINVAL;
    const uint32_t n = h.n_records;
    if (!n) {
        if (first_shard) *first_shard = opts.records_per_shard == 0 ? 0u : (uint32_t)shards.size();
        return PX_OK;
    }
    // ---- bytes to the device (one store allocation: data, then lane entries)
    auto *d_src = (uint8_t **)heap.alloc((uint64_t)n * 8);
    auto *d_len = (uint32_t *)heap.alloc((uint64_t)n * 8);
    uint32_t *d_nesc = d_len + n;
    const uint64_t data_cap = round_up(h.data_bytes + 64, 16);
    // lane entries need the 251 counts: stage the data first, count, then size the rest
    auto *data = (uint8_t *)heap.alloc(data_cap);
    if (src_on_device)
        hcheck(hipMemcpyAsync(data, src + h.data_off, h.data_bytes, hipMemcpyDeviceToDevice, stream));
    else
        h2d_bulk(data, src + h.data_off, h.data_bytes);
    std::vector<uint8_t *> sp(n);
    std::vector<uint32_t> cl(n);
    for (uint32_t i = 0; i < n; ++i) {
        sp[i] = data + br[i].off;
        cl[i] = br[i].comp_len;
    }
    h2d(d_src, sp.data(), (size_t)n * 8);
    h2d(d_len, cl.data(), (size_t)n * 4);
    hcheck(launch_count_esc(stream, n, d_src, d_len, d_nesc));
    std::vector<uint32_t> nesc(n);
    d2h(nesc.data(), d_nesc, (size_t)n * 4);
    sync();
    heap.release(d_src, (uint64_t)n * 8);
    heap.release(d_len, (uint64_t)n * 8);
    std::vector<uint64_t> soff(n + 1, 0), poff(n + 1, 0);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t dl = br[i].doc_len & ~kBlobDead;
        soff[i + 1] = soff[i] + seg_entries(nesc[i]) * sizeof(SegEnt);
        poff[i + 1] = poff[i] + round_up(pidx_blocks(dl) * 2, 16);
    }
    // the store keeps data and lane entries in one allocation (LaneEnt::rel is relative)
    const uint64_t lane_at = data_cap, store_bytes = lane_at + soff[n] + 64;  // (LaneEnt: the size of a SegEnt)
    auto *store = (uint8_t *)store_alloc(store_bytes);
    hcheck(hipMemcpyAsync(store, data, h.data_bytes, hipMemcpyDeviceToDevice, stream));
    auto *segs = (uint8_t *)heap.alloc(soff[n] + poff[n] + 64);
    store_blocks.emplace_back(store, store_bytes);
    store_blocks.emplace_back(segs, soff[n] + poff[n] + 64);
    macct.comp += lane_at;
    macct.lane += soff[n] + 64;
    macct.seg += soff[n];
    macct.pidx += poff[n] + 64;
    std::vector<RecSlot> slots(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t dl = br[i].doc_len & ~kBlobDead;
        slots[i] = RecSlot{store + br[i].off, (const SegEnt *)(segs + soff[i]),
                           (const uint16_t *)(segs + soff[n] + poff[i]), br[i].comp_len, 0, pidx_blocks(dl), 0,
                           (const LaneEnt *)(store + lane_at + soff[i])};
    }
    auto *d_slots = (RecSlot *)heap.alloc((uint64_t)n * sizeof(RecSlot));
    auto *d_tmp = (uint32_t *)heap.alloc((uint64_t)n * 8);
    h2d(d_slots, slots.data(), (size_t)n * sizeof(RecSlot));
    hcheck(launch_tokenize(stream, n, d_slots, d_tmp, d_tmp + n, nullptr));
    std::vector<uint32_t> nseg(n), tst(n);
    d2h(nseg.data(), d_tmp, (size_t)n * 4);
    d2h(tst.data(), d_tmp + n, (size_t)n * 4);
    sync();
    heap.release(data, data_cap);
    heap.release(d_slots, (uint64_t)n * sizeof(RecSlot));
    heap.release(d_tmp, (uint64_t)n * 8);
    // ---- shards and chunks (a single-shard store takes them into shard 0, empty or new)
    const uint32_t first = opts.records_per_shard == 0 ? 0u : (uint32_t)shards.size();
    std::map<uint32_t, Shard *> target;  // source shard -> shard here
    std::vector<uint32_t> rchunk(n);
    std::vector<Shard *> rshard(n);
    for (const BlobChunk &c : bc) {
        Shard *s;
        if (opts.records_per_shard == 0) {
            s = shards.empty() ? &new_shard() : shards[0].get();
        } else {
            auto it = target.find(c.shard);
            s = it != target.end() ? it->second : (target[c.shard] = &new_shard());
        }
        const uint32_t g = new_chunk(s->id);
        s->chunks.push_back(g);
        Chunk &ch = chunks[g];
        for (uint32_t i = c.first; i < c.first + c.n; ++i) {
            set_nseg(slots[i], nseg[i]);
            ch.slots.push_back(slots[i]);
            ch.doc_len.push_back(br[i].doc_len & ~kBlobDead);
            ch.dead.push_back((br[i].doc_len & kBlobDead) || tst[i] != kOk ? 1 : 0);
            ch.kp_off.push_back(0);
            ch.kp_len.push_back(0);
            rchunk[i] = g;
            rshard[i] = s;
        }
        ch.n = c.n;
        for (uint32_t i = 0; i < c.n; ++i) ch.used += ch.dead[i] ? 0 : 1;
        ch.total = c.n;  // a loaded chunk is closed
        s->records += c.n;
        // the next set batch starts this shard's GST in a fresh chunk after the loaded ones
        s->hs.chunk_seq = (uint32_t)s->chunks.size();
        chunk_reserve(g, c.n);
        h2d(ch.dev, ch.slots.data(), (size_t)c.n * sizeof(RecSlot));
    }
    if (opts.records_per_shard != 0)  // new records go to new shards, never into a loaded one
        for (auto &t : target) t.second->records = std::max(t.second->records, opts.records_per_shard);
    {
        std::vector<LinkJob> jobs;
        for (const BlobChunk &c : bc) {
            const uint32_t g = rchunk[c.first];
            for (uint32_t i = 0; i < c.n; ++i) {
                const RecSlot &sl = chunks[g].slots[i];
                jobs.push_back(LinkJob{const_cast<SegEnt *>(sl.seg), const_cast<LaneEnt *>(sl.lane), chunks[g].dev,
                                       sl.nseg, c.n});
            }
        }
        link(jobs);
    }
    // ---- index the live records: compat key prefixes, then CritBit (and the key map)
    std::vector<KpJob> jobs;
    std::vector<uint32_t> jrec;
    for (const BlobChunk &c : bc)
        for (uint32_t k = 0; k < c.n; ++k) {
            const uint32_t i = c.first + k;
            if (chunks[rchunk[i]].dead[k]) continue;
            const uint32_t dl = br[i].doc_len & ~kBlobDead;
            jobs.push_back(KpJob{rchunk[i], k, dl, std::min<uint32_t>(dl + 64, 576)});
            jrec.push_back(i);
        }
    std::vector<uint32_t> kst;
    decode_key_prefixes(jobs, kst);
    int rc = PX_OK;
    for (size_t j = 0; j < jobs.size(); ++j) {
        Chunk &ch = chunks[jobs[j].chunk];
        const uint32_t k = jobs[j].idx;
        uint32_t kl = 0;
        const uint8_t *kp = kp_of(Leaf{jobs[j].chunk, k}, &kl);
        if (kst[j] != kOk || kl < 2 || kp[kl - 2] != kEsc || kp[kl - 1] != kKeyEnd) {
            if (!ch.dead[k] && ch.used) ch.used--;
            ch.dead[k] = 1;  // no decodable key: not indexed
            if (rc == PX_OK) rc = kst[j] != kOk ? (int)map_status(kst[j]) : PX_ECORRUPT;
            continue;
        }
        Shard &s = *rshard[jrec[j]];
        std::string q(reinterpret_cast<const char *>(kp), kl);
        if (opts.records_per_shard != 0) {
            std::string raw;  // the raw key: the escaped prefix without 251,0, 251 pairs undoubled
            for (uint32_t b = 0; b + 2 < kl + 0u; ++b) {
                raw.push_back((char)kp[b]);
                if (kp[b] == kEsc) ++b;
            }
            const auto *rk = reinterpret_cast<const uint8_t *>(raw.data());
            const int64_t prev = keymap.find(rk, raw.size());
            if (prev >= 0 && (uint32_t)prev != s.id) cbt_delete(*shards[(size_t)prev], q);
            keymap.put(rk, raw.size(), s.id, jobs[j].chunk, k);
        }
        (void)cbt_insert(s, q, Leaf{jobs[j].chunk, k});  // (1: a duplicate key inside the blob replaced the earlier)
    }
    // span tables for the loaded records (compat only: without their docs compat == exact is
    // unknown, so exact getitems of loaded records keep the segment walk)
    {
        std::vector<SpanReq> reqs;
        for (const BlobChunk &c : bc)
            for (uint32_t k = 0; k < c.n; ++k)
                if (!chunks[rchunk[c.first + k]].dead[k]) reqs.push_back(SpanReq{rchunk[c.first + k], k, nullptr});
        build_spans(reqs, 0, false);
    }
    stats.chunks = chunks.size();
    if (first_shard) *first_shard = first;
    return rc;
}

// ====================================================================== C ABI
extern "C" {

// Host heap policy (once per process, PX_NO_MALLOPT=1 leaves glibc's defaults): a set batch
// of a million records builds ~1 GB of per-record host arrays, and glibc serves each array
// over 32 MB -- and, past its dynamic threshold, smaller ones -- by a fresh mmap that it
// unmaps at free, so every batch paid first-touch page faults on all of them again (config 4:
// 244 -> 177 ms per set batch with the policy, profiles/r06c_cfg4_set_phases_*.log).  With mmap off and
// the trim threshold out of reach, freed blocks stay in the heap and the next batch reuses
// pages already mapped.  The cost: the process keeps its host heap's high-water mark.
static void host_heap_policy() {
    static std::once_flag once;
    std::call_once(once, [] {
        const char *e = std::getenv("PX_NO_MALLOPT");
        if (e && e[0] == '1') return;
        mallopt(M_MMAP_MAX, 0);
        mallopt(M_TRIM_THRESHOLD, 0x7fffffff);
    });
}

px_ctx *px_open(const px_opts *opts) {
    try {
        host_heap_policy();
        auto *c = new px_ctx();
        if (opts) c->opts = *opts;
        hcheck(hipSetDevice(c->opts.device));
        hcheck(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        hcheck(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
        hcheck(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
        hcheck(hipEventCreate(&c->ev0));
        hcheck(hipEventCreate(&c->ev1));
        hcheck(hipEventCreate(&c->ev_mid));
        hcheck(hipEventCreateWithFlags(&c->ev_get, hipEventDisableTiming));
        return c;
    } catch (...) {
        return nullptr;
    }
}

void px_close(px_ctx *ctx) {
    if (!ctx) return;
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->ev_mid) (void)hipEventDestroy(ctx->ev_mid);
    if (ctx->ev_get) (void)hipEventDestroy(ctx->ev_get);
    for (auto &e : ctx->ring_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream2) {
        (void)hipStreamSynchronize(ctx->stream2);
        (void)hipStreamDestroy(ctx->stream2);
    }
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *px_strerror(int s) {
    switch (s) {
    case PX_OK: return "ok";
    case PX_EINVAL: return "invalid argument (empty key or escaped doc > 65535 bytes)";
    case PX_ECAPACITY: return "internal arena capacity exceeded";
    case PX_EREFCRASH: return "input on which the reference GST dereferences NULL";
    case PX_ECORRUPT: return "malformed compressed bytes";
    case PX_EHANG: return "input on which the reference decoder never terminates";
    case PX_EDEPTH: return "decode nesting exceeds decode_depth";
    case PX_ESPACE: return "output buffer too small";
    case PX_ENOTFOUND: return "key not found";
    case PX_EHIP: return "HIP runtime error";
    case PX_ENOMEM: return "device allocation failed";
    default: return "unknown status";
    }
}

#define PX_GUARD(...)                                    \
    try {                                                \
        __VA_ARGS__                                      \
    } catch (const HipFail &f) {                         \
        ctx->last_hip = (int)f.e;                        \
        fprintf(stderr, "pixiu_amd: HIP error %s at px_runtime.cpp:%d\n", hipGetErrorName(f.e), f.line); \
        return PX_EHIP;                                  \
    } catch (const PxFail &f) {                          \
        return f.code;                                   \
    } catch (const std::bad_alloc &) {                   \
        return PX_ENOMEM;                                \
    }

// every call but px_set_batch / px_flush / px_reset / px_close stores the write-behind
// queue first, so reads see every record set before them
#define PX_FLUSHED(ctx) (void)(ctx)->flush_queue()

int px_set_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, const uint8_t *vals,
                 const uint64_t *voff, int on_device, px_set_result *res) {
    if (!ctx || (n && (!keys || !koff || !voff))) return PX_EINVAL;
    PX_GUARD({
        if (ctx->defer_on() && !on_device && n && n <= 64)
            return ctx->set_deferred(n, keys, koff, vals, voff, res);
        PX_FLUSHED(ctx);
        const int rc = ctx->set_ctrl(n, keys, koff, vals, voff, on_device, res);
        ctx->note_last(n, res);
        return rc;
    })
}

int px_set_docs(px_ctx *ctx, uint32_t n, const uint8_t *docs, const uint64_t *doff, int on_device, int reinsert,
                px_set_result *res) {
    if (!ctx || (n && (!docs || !doff))) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        std::vector<uint64_t> zero(n + 1, 0);
        uint8_t dummy = 0;
        struct Raw {  // raw_docs for the duration of the call, restored on every exit
            px_ctx *c;
            bool saved;
            ~Raw() { c->raw_docs = saved; }
        } raw{ctx, ctx->raw_docs};
        ctx->raw_docs = true;
        int rc = PX_OK;
        if (!reinsert || ctx->opts.records_per_shard != 0) {
            // (the Glob_Reinsert_Chunk trigger only exists for the single instance)
            rc = ctx->set_ctrl(n, docs, doff, &dummy, zero.data(), on_device, res);
        } else {
            // setitem(doc, reinsert = true): the rotation trigger only (PiXiuCtrl.cpp:13-29),
            // evaluated before every record as reinsert_chunk does
            std::vector<uint64_t> ho(n + 1);
            if (on_device) {
                ctx->d2h(ho.data(), doff, (size_t)(n + 1) * 8);
                ctx->sync();
            } else {
                std::memcpy(ho.data(), doff, (size_t)(n + 1) * 8);
            }
            for (uint32_t pos = 0; pos < n;) {
                Shard *s = ctx->shards.empty() ? nullptr : ctx->shards[0].get();
                uint32_t end = n;
                if (s) {
                    ctx->reinsert_triggers(*s, px_ctx::kTrigReinsert);
                    const uint32_t room = (uint32_t)kChunkSlots - std::min<uint32_t>(s->hs.n_docs, kChunkSlots);
                    end = std::min(n, pos + std::max(room, 1u));
                }
                const int r2 = ctx->set_batch(end - pos, docs, ho.data() + pos, &dummy, zero.data(), on_device,
                                              res ? res + pos : nullptr);
                if (rc == PX_OK) rc = r2;
                pos = end;
            }
        }
        ctx->note_last(n, res);
        return rc;
    })
}

int px_flush(px_ctx *ctx, px_set_result *last) {
    if (!ctx) return PX_EINVAL;
    // the failure is handed out once: dq_rc is cleared whether the flush itself threw or not
    // (a failed flush_queue() records its code there too)
    const int rc = [&]() -> int {
        PX_GUARD({
            ctx->flush_queue();
            if (last && ctx->have_last) *last = ctx->last_res;
            return PX_OK;
        })
    }();
    const int dq = ctx->dq_rc;
    ctx->dq_rc = PX_OK;
    return rc != PX_OK ? rc : dq;
}

static int get_batch_impl(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, int mode, uint8_t *out,
                          uint64_t out_cap, int out_on_device, uint64_t *out_off, uint32_t *out_len, uint32_t *status,
                          uint64_t *needed, bool try_device) {
    const auto t0 = std::chrono::steady_clock::now();
    int rc;
    double lookup_ms = 0;
    ctx->stats.last_get_device_keys = 0;
    rc = ctx->opts.decode_waves == 0 && try_device
             ? ctx->dki_get(n, keys, koff, mode, out, out_cap, out_on_device, out_off, out_len, status, needed)
             : -1;
    const bool on_device = rc != -1;
    if (on_device) {
        // (resolved on the device: no host lookups; rc is the first failing status)
    } else if (out_on_device && n >= 4096 && ctx->opts.decode_waves == 0) {
        rc = ctx->get_overlapped(n, keys, koff, mode, out, out_cap, out_off, out_len, status, needed, lookup_ms);
    } else {
        std::vector<DecodeQuery> q(n);
        std::vector<uint32_t> pre(n, PX_OK);
        // key -> record lookups are read-only: host threads over key ranges
        parallel_ranges(n, ctx->host_threads(), [&](uint32_t lo, uint32_t hi) {
            std::string ek;
            for (uint32_t i = lo; i < hi; ++i)
                ctx->resolve_key(keys + koff[i], koff[i + 1] - koff[i], mode, ek, q[i], pre[i]);
        });
        lookup_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        rc = ctx->expand(q, out, out_cap, out_on_device, out_off, out_len, status, needed, pre);
    }
    if (rc == PX_OK && !on_device)
        for (uint32_t i = 0; i < n; ++i)
            if (status[i] != PX_OK) {
                rc = (int)status[i];
                break;
            }
    ctx->stats.last_get_lookup_ms = lookup_ms;
    ctx->stats.last_get_call_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int px_get_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, int mode, uint8_t *out,
                 uint64_t out_cap, int out_on_device, uint64_t *out_off, uint32_t *out_len, uint32_t *status,
                 uint64_t *needed) {
    if (!ctx || (n && (!keys || !koff || !out_off || !out_len || !status))) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        return get_batch_impl(ctx, n, keys, koff, mode, out, out_cap, out_on_device, out_off, out_len, status, needed,
                              true);
    })
}

int px_get_batch_dev(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, int mode, uint8_t *out,
                     uint64_t out_cap, uint64_t *out_off, uint32_t *out_len, uint32_t *status, uint64_t *needed) {
    if (!ctx || (n && (!keys || !koff || !out || !out_off || !out_len || !status))) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        if (needed) *needed = 0;
        if (!n) return PX_OK;
        const auto t0 = std::chrono::steady_clock::now();
        ctx->stats.last_get_device_keys = 0;
        int rc = ctx->opts.decode_waves == 0 ? ctx->dki_get(n, keys, koff, mode, out, out_cap, 1, out_off, out_len,
                                                             status, needed, true)
                                             : -1;
        if (rc == -1) {
            // keys the device index does not answer: keys and offsets down, the host path, the
            // results up (offsets rebased to the first key)
            std::vector<uint64_t> ko(n + 1);
            ctx->d2h(ko.data(), koff, (size_t)(n + 1) * 8);
            ctx->sync();
            const uint64_t k0 = ko[0];
            std::vector<uint8_t> kb(ko[n] - k0 + 1);
            if (ko[n] > k0) ctx->d2h(kb.data(), keys + k0, ko[n] - k0);
            ctx->sync();
            for (auto &x : ko) x -= k0;
            std::vector<uint64_t> ho(n);
            std::vector<uint32_t> hl(n), hs(n);
            rc = get_batch_impl(ctx, n, kb.data(), ko.data(), mode, out, out_cap, 1, ho.data(), hl.data(), hs.data(),
                                needed, false);
            ctx->h2d(out_off, ho.data(), (size_t)n * 8);
            ctx->h2d(out_len, hl.data(), (size_t)n * 4);
            ctx->h2d(status, hs.data(), (size_t)n * 4);
            ctx->sync();
        }
        ctx->stats.last_get_call_ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return rc;
    })
}

int px_parse_batch(px_ctx *ctx, uint32_t n, const px_rec *recs, int mode, uint8_t *out, uint64_t out_cap,
                   int out_on_device, uint64_t *out_off, uint32_t *out_len, uint32_t *status, uint64_t *needed) {
    if (!ctx || (n && (!recs || !out_off || !out_len || !status))) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        std::vector<DecodeQuery> q(n);
        std::vector<uint32_t> pre(n, PX_OK);
        for (uint32_t i = 0; i < n; ++i) {
            const px_rec &r = recs[i];
            q[i] = DecodeQuery{kNone, 0, r.from, r.to, 0, 0, (uint32_t)mode};
            if (r.shard >= ctx->shards.size() || r.chunk >= ctx->shards[r.shard]->chunks.size() ||
                r.from < 0 || r.to < r.from) {
                pre[i] = PX_EINVAL;
                continue;
            }
            uint32_t c = ctx->shards[r.shard]->chunks[r.chunk];
            if (r.idx >= ctx->chunks[c].n) {
                pre[i] = PX_EINVAL;
                continue;
            }
            q[i].chunk = c;
            q[i].idx = r.idx;
            uint64_t span = std::min<uint64_t>((uint64_t)(r.to - r.from), ctx->chunks[c].doc_len[r.idx]);
            q[i].out_cap = (uint32_t)round_up(span + 64, 16);
        }
        return ctx->expand(q, out, out_cap, out_on_device, out_off, out_len, status, needed, pre);
    })
}

int px_locate_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, px_rec *recs,
                    uint32_t *status) {
    if (!ctx || (n && (!keys || !koff || !recs || !status))) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        std::string ek;
        for (uint32_t i = 0; i < n; ++i) {
            DecodeQuery q;
            uint32_t pre = PX_OK;
            ctx->resolve_key(keys + koff[i], koff[i + 1] - koff[i], PX_COMPAT, ek, q, pre);
            status[i] = pre;
            recs[i] = px_rec{0, 0, 0, 0, kMaxDoc};
            if (pre != PX_OK) continue;
            const uint32_t sh = ctx->chunks[q.chunk].shard;
            const auto &cs = ctx->shards[sh]->chunks;
            recs[i].shard = sh;
            recs[i].chunk = (uint32_t)(std::find(cs.begin(), cs.end(), q.chunk) - cs.begin());
            recs[i].idx = q.idx;
        }
        return PX_OK;
    })
}

int px_reinsert(px_ctx *ctx, uint32_t shard, uint32_t chunk) {
    if (!ctx || shard >= ctx->shards.size()) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        Shard &s = *ctx->shards[shard];
        if (chunk >= s.chunks.size()) return PX_EINVAL;
        const uint32_t c = s.chunks[chunk];
        const Chunk &ch = ctx->chunks[c];
        // closed (PiXiuChunk::total_num set at rotation) and slot-full; the live chunk is the
        // shard's last one
        if (chunk + 1 == s.chunks.size() || ch.total == 0 || ch.n != (uint32_t)kChunkSlots || ch.used == 0)
            return PX_EINVAL;  // (used 0: compacted already -- the reference's pointer is NULL by then)
        ctx->reinsert_chunk(s, c, false);
        if (s.glob == (int64_t)c) s.glob = -1;  // (the reference would keep a dangling Glob_Reinsert_Chunk)
        return PX_OK;
    })
}

int px_contains_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, uint32_t *result) {
    if (!ctx || (n && (!keys || !koff || !result))) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        for (uint32_t i = 0; i < n; ++i) {
            Shard *s = ctx->shard_for_key(keys + koff[i], koff[i + 1] - koff[i]);
            result[i] = s && ctx->cbt_contains(*s, px_ctx::esc_key(keys + koff[i], koff[i + 1] - koff[i]));
        }
        return PX_OK;
    })
}

int px_del_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, uint32_t *result) {
    if (!ctx || (n && (!keys || !koff || !result))) return PX_EINVAL;
    PX_GUARD(PX_FLUSHED(ctx); return ctx->del_ctrl(n, keys, koff, result);)
}

int px_iter(px_ctx *ctx, const uint8_t *prefix, uint64_t prefix_len, px_rec *recs, uint32_t cap, uint32_t *n_out) {
    if (!ctx || !n_out || (prefix_len && !prefix) || (cap && !recs)) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        std::string p;  // PiXiuStr_init: 251 doubled, no terminator
        for (uint64_t i = 0; i < prefix_len; ++i) {
            p.push_back((char)prefix[i]);
            if (prefix[i] == kEsc) p.push_back((char)kEsc);
        }
        std::vector<px_rec> got;
        bool any_tree = false;
        for (auto &sp : ctx->shards) {
            std::vector<Leaf> leaves;
            if (!ctx->cbt_iter(*sp, p, leaves)) continue;
            any_tree = true;
            std::unordered_map<uint32_t, uint32_t> seq;
            for (uint32_t k = 0; k < sp->chunks.size(); ++k) seq[sp->chunks[k]] = k;
            for (const Leaf &l : leaves) got.push_back(px_rec{sp->id, seq[l.chunk], l.idx, 0, kMaxDoc});
        }
        *n_out = (uint32_t)got.size();
        if (!any_tree) return PX_ENOTFOUND;
        if (got.size() > cap) return PX_ESPACE;
        if (!got.empty()) memcpy(recs, got.data(), got.size() * sizeof(px_rec));
        return PX_OK;
    })
}

int px_export(px_ctx *ctx, uint32_t n, const px_rec *recs, uint8_t *out, uint64_t out_cap, uint64_t *out_off) {
    if (!ctx || (n && (!recs || !out_off))) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        out_off[0] = 0;
        for (uint32_t i = 0; i < n; ++i) {
            const px_rec &r = recs[i];
            if (r.shard >= ctx->shards.size() || r.chunk >= ctx->shards[r.shard]->chunks.size()) return PX_EINVAL;
            const Chunk &ch = ctx->chunks[ctx->shards[r.shard]->chunks[r.chunk]];
            if (r.idx >= ch.n) return PX_EINVAL;
            const RecSlot &sl = ch.slots[r.idx];
            if (out_off[i] + sl.comp_len > out_cap) return PX_ESPACE;
            ctx->d2h(out + out_off[i], sl.comp, sl.comp_len);
            out_off[i + 1] = out_off[i] + sl.comp_len;
        }
        ctx->sync();
        return PX_OK;
    })
}

int px_last_store(px_ctx *ctx, uint8_t *dst, uint64_t cap, int dst_on_device, uint64_t *bytes) {
    if (!ctx) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        if (bytes) *bytes = ctx->last_store_bytes;
        if (!dst) return PX_OK;
        if (cap < ctx->last_store_bytes) return PX_ESPACE;
        if (ctx->last_store_bytes && dst_on_device)
            hcheck(hipMemcpyAsync(dst, ctx->last_store, ctx->last_store_bytes, hipMemcpyDeviceToDevice, ctx->stream));
        else
            ctx->d2h(dst, ctx->last_store, ctx->last_store_bytes);
        ctx->sync();
        return PX_OK;
    })
}

// Import a chunk of compressed records (e.g. exported earlier, or hand-built for the
// decoder known-answer tests) as a new read-only shard; returns its shard id.
int px_import_chunk(px_ctx *ctx, uint32_t n, const uint8_t *comp, const uint64_t *off, uint32_t *shard_out) {
    if (!ctx || !n || n > (uint32_t)kChunkSlots || !comp || !off) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        // an imported record's source length is unknown up front: index the first
        // kMaxDoc source bytes (a lane asking past that goes to the serial path)
        const uint32_t pn = pidx_blocks(kMaxDoc);
        std::vector<uint64_t> coff(n + 1, 0), soff(n + 1, 0), nents(n);
        for (uint32_t r = 0; r < n; ++r) {
            uint64_t l = off[r + 1] - off[r];
            if (l > (uint64_t)kMaxDoc) return PX_EINVAL;
            uint64_t esc = 0;
            for (uint64_t i = off[r]; i < off[r + 1]; ++i) esc += comp[i] == kEsc;
            nents[r] = seg_entries((uint32_t)esc);
            coff[r + 1] = coff[r] + round_up(l, 8);
            soff[r + 1] = soff[r] + nents[r] * sizeof(SegEnt) + round_up((uint64_t)pn * 2, 16);
        }
        std::vector<uint64_t> loff(n + 1, 0);
        for (uint32_t r = 0; r < n; ++r) loff[r + 1] = loff[r] + nents[r] * sizeof(LaneEnt);
        const uint64_t lane_at = round_up(coff[n] + 64, 16), store_bytes = lane_at + loff[n] + 64;
        auto *store = (uint8_t *)ctx->store_alloc(store_bytes);
        auto *segs = (uint8_t *)ctx->heap.alloc(soff[n] + 64);
        ctx->store_blocks.emplace_back(store, store_bytes);
        ctx->store_blocks.emplace_back(segs, soff[n] + 64);
        std::vector<RecSlot> slots(n);
        for (uint32_t r = 0; r < n; ++r) {
            uint64_t l = off[r + 1] - off[r];
            ctx->h2d(store + coff[r], comp + off[r], l);
            slots[r] = RecSlot{store + coff[r], (const SegEnt *)(segs + soff[r]),
                               (const uint16_t *)(segs + soff[r] + nents[r] * sizeof(SegEnt)), (uint32_t)l, 0, pn, 0,
                               (const LaneEnt *)(store + lane_at + loff[r])};
        }
        auto *d_slots = (RecSlot *)ctx->heap.alloc((uint64_t)n * sizeof(RecSlot));
        auto *d_tmp = (uint32_t *)ctx->heap.alloc((uint64_t)n * 8);
        ctx->h2d(d_slots, slots.data(), (size_t)n * sizeof(RecSlot));
        hcheck(launch_tokenize(ctx->stream, n, d_slots, d_tmp, d_tmp + n, nullptr));
        std::vector<uint32_t> nseg(n), tst(n);
        ctx->d2h(nseg.data(), d_tmp, (size_t)n * 4);
        ctx->d2h(tst.data(), d_tmp + n, (size_t)n * 4);
        ctx->sync();
        std::vector<SegEnt> sentinel(n);
        for (uint32_t r = 0; r < n; ++r) ctx->d2h(&sentinel[r], slots[r].seg + (nseg[r] & ~kNoPidxBit), sizeof(SegEnt));
        ctx->sync();
        ctx->heap.release(d_slots, (uint64_t)n * sizeof(RecSlot));
        ctx->heap.release(d_tmp, (uint64_t)n * 8);
        for (uint32_t r = 0; r < n; ++r)
            if (tst[r] != kOk) return (int)map_status(tst[r]);
        Shard &sh = ctx->new_shard();
        sh.records = n;
        uint32_t c = ctx->new_chunk(sh.id);
        sh.chunks.push_back(c);
        Chunk &ch = ctx->chunks[c];
        for (uint32_t r = 0; r < n; ++r) {
            set_nseg(slots[r], nseg[r]);
            ch.slots.push_back(slots[r]);
            ch.doc_len.push_back(std::min<uint32_t>(sentinel[r].x, (uint32_t)kMaxDoc * 4));
            ch.dead.push_back(0);
            ch.kp_off.push_back(0);
            ch.kp_len.push_back(0);
        }
        ch.n = n;
        ctx->chunk_reserve(c, n);
        ctx->h2d(ctx->chunks[c].dev, ctx->chunks[c].slots.data(), (size_t)n * sizeof(RecSlot));
        std::vector<LinkJob> jobs(n);
        for (uint32_t r = 0; r < n; ++r)
            jobs[r] = LinkJob{const_cast<SegEnt *>(ctx->chunks[c].slots[r].seg),
                              const_cast<LaneEnt *>(ctx->chunks[c].slots[r].lane), ctx->chunks[c].dev,
                              ctx->chunks[c].slots[r].nseg, n};
        ctx->link(jobs);
        ctx->sync();
        if (shard_out) *shard_out = sh.id;
        return PX_OK;
    })
}

int px_save(px_ctx *ctx, uint8_t *dst, uint64_t cap, int dst_on_device, uint64_t *bytes) {
    if (!ctx) return PX_EINVAL;
    PX_GUARD(PX_FLUSHED(ctx); return ctx->save(dst, cap, dst_on_device, bytes);)
}

int px_load(px_ctx *ctx, const uint8_t *src, uint64_t len, int src_on_device, uint32_t *first_shard) {
    if (!ctx || (len && !src)) return PX_EINVAL;
    // (loaded records move the key map's hints; the device key index does not follow them)
    PX_GUARD(PX_FLUSHED(ctx); ctx->dki.valid = false; ctx->dki_clear();
             return ctx->load(src, len, src_on_device, first_shard);)
}

int px_reset(px_ctx *ctx) {
    if (!ctx) return PX_EINVAL;
    PX_GUARD(ctx->drop_queue(); ctx->have_last = false; ctx->dq_rc = PX_OK; ctx->reset(); return PX_OK;)
}

int px_stats_get(px_ctx *ctx, px_stats *st) {
    if (!ctx || !st) return PX_EINVAL;
    PX_GUARD({
        PX_FLUSHED(ctx);
        *st = ctx->stats;
        st->device_bytes = ctx->heap.held() + ctx->arena.mapped;
        st->device_live_bytes = ctx->heap.live_bytes() + ctx->arena.top;
        st->device_peak_bytes = ctx->heap.peak();
        ctx->mem_stats(st);
        return PX_OK;
    })
}

int px_trim(px_ctx *ctx, uint64_t keep_bytes) {
    if (!ctx) return PX_EINVAL;
    PX_GUARD({
        ctx->sync();
        ctx->heap.trim(keep_bytes);
        ctx->stats.device_bytes = ctx->heap.held() + ctx->arena.mapped;
        return PX_OK;
    })
}

void *px_stream(px_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

// debug builds (make trace): per-byte encoder messages of the first shard of the last batch
int px_debug_trace_take(int32_t *out, uint32_t cap) { return px::debug_trace_take(out, cap); }
// debug builds (make prof): k_gst_encode counters/cycles accumulated since the last call
int px_debug_prof_take(unsigned long long *out, uint32_t cap) { return px::debug_prof_take(out, cap); }

}  // extern "C"
