// px_host.h — the host-only parts of the runtime (no HIP): the CritBit index the north
// star keeps on the host, the key -> shard maps, the worker pool, the best-fit block heap
// (over any raw allocator), and the per-phase clock.  px_runtime.cpp instantiates them
// over device memory and the GPU-decoded key prefixes; tests/cpp/host_test.cpp runs the
// same code on the CPU under AddressSanitizer / UndefinedBehaviorSanitizer.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace pxh {

constexpr uint8_t kEscByte = 251;    // PXS_UNIQUE (PiXiuStr.h:11-21)
constexpr uint8_t kKeyEndByte = 0;   // PXS_KEY

inline uint64_t round_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// ---------------------------------------------------------------- block heap
// Best-fit allocator over slabs from a raw allocator (Raw::get(bytes) -> pointer or null,
// Raw::put(pointer)): a free block is split on allocation and merged with its free
// neighbours (inside its slab) on release, so batches of varying sizes reuse the same
// memory instead of growing the footprint.  alloc() returns null when Raw fails.
template <class Raw>
class BlockHeap {
  public:
    explicit BlockHeap(uint64_t slab = 1ull << 30) : slab_(slab) {}
    BlockHeap(const BlockHeap &) = delete;
    ~BlockHeap() {
        for (auto &s : slabs_) Raw::put(s.first);
    }
    void *alloc(uint64_t n) {
        n = round_up(std::max<uint64_t>(n, 256), 256);
        auto it = by_size_.lower_bound(n);
        if (it == by_size_.end()) {
            const uint64_t sz = std::max<uint64_t>(n, slab_);
            char *s = static_cast<char *>(Raw::get(sz));
            if (!s) return nullptr;
            slabs_.emplace(s, s + sz);
            held_ += sz;
            peak_ = std::max(peak_, held_);
            add_free(s, sz);
            it = by_size_.lower_bound(n);
        }
        char *p = it->second;
        uint64_t sz = it->first;
        by_size_.erase(it);
        by_addr_.erase(p);
        if (sz - n >= 256) {  // split: the tail stays free
            add_free(p + n, sz - n);
            sz = n;
        }
        live_[p] = sz;
        live_total_ += sz;
        live_peak_ = std::max(live_peak_, live_total_);
        return p;
    }
    void release(void *v) {
        if (!v) return;
        char *p = static_cast<char *>(v);
        auto lv = live_.find(p);
        if (lv == live_.end()) return;
        uint64_t sz = lv->second;
        live_.erase(lv);
        live_total_ -= sz;
        auto slab = std::prev(slabs_.upper_bound(p));  // the slab holding p
        // merge with the free block right after and right before, inside the slab
        auto nx = by_addr_.find(p + sz);
        if (nx != by_addr_.end() && nx->first < slab->second) {
            sz += nx->second;
            erase_free(nx->first, nx->second);
        }
        auto pv = by_addr_.lower_bound(p);
        if (pv != by_addr_.begin()) {
            --pv;
            if (pv->first >= slab->first && pv->first + pv->second == p) {
                char *q = pv->first;
                const uint64_t qs = pv->second;
                erase_free(q, qs);
                p = q;
                sz += qs;
            }
        }
        add_free(p, sz);
    }
    uint64_t held() const { return held_; }
    uint64_t peak() const { return peak_; }
    // Give wholly free slabs back to Raw (largest first) until the free bytes cached in
    // the slabs still held are <= keep; returns the bytes given back.
    uint64_t trim(uint64_t keep) {
        uint64_t free_b = cached_free(), back = 0;
        if (free_b <= keep) return 0;
        std::vector<std::pair<uint64_t, char *>> whole;  // (size, start) of wholly free slabs
        for (const auto &s : slabs_) {
            auto f = by_addr_.find(s.first);
            if (f != by_addr_.end() && f->second == (uint64_t)(s.second - s.first)) whole.emplace_back(f->second, s.first);
        }
        std::sort(whole.begin(), whole.end(), [](const auto &a, const auto &b) { return a.first > b.first; });
        for (const auto &w : whole) {
            if (free_b <= keep) break;
            erase_free(w.second, w.first);
            slabs_.erase(w.second);
            Raw::put(w.second);
            held_ -= w.first;
            free_b -= w.first;
            back += w.first;
        }
        return back;
    }
    uint64_t cached_free() const {  // bytes in free blocks of the slabs already held
        uint64_t f = 0;
        for (const auto &b : by_addr_) f += b.second;
        return f;
    }
    uint64_t live_bytes() const { return live_total_; }
    // the most bytes live at once since the last mark_peak() (a set batch's scratch peak)
    uint64_t live_peak() const { return live_peak_; }
    void mark_peak() { live_peak_ = live_total_; }

  private:
    void add_free(char *p, uint64_t sz) {
        by_addr_[p] = sz;
        by_size_.emplace(sz, p);
    }
    void erase_free(char *p, uint64_t sz) {
        by_addr_.erase(p);
        for (auto r = by_size_.equal_range(sz); r.first != r.second; ++r.first)
            if (r.first->second == p) {
                by_size_.erase(r.first);
                break;
            }
    }
    uint64_t slab_;
    std::map<char *, char *> slabs_;  // start -> end
    std::map<char *, uint64_t> by_addr_;
    std::multimap<uint64_t, char *> by_size_;
    std::unordered_map<void *, uint64_t> live_;
    uint64_t held_ = 0, peak_ = 0;
    uint64_t live_total_ = 0, live_peak_ = 0;
};

// ---------------------------------------------------------------- key maps
// raw key -> shard for multi-shard stores.  Open addressing over 64-bit key hashes
// with the key bytes in one arena: a lookup touches one slot and the key's bytes,
// with no per-key heap node and no std::string built for the probe.
class KeyMap {
    struct Slot {
        uint64_t h, off;
        uint32_t len, shard;  // len == kFree: empty
        uint32_t chunk, idx;  // the record last stored under the key (a hint: verified on use)
    };
    static constexpr uint32_t kFree = ~0u;
    std::vector<Slot> tab_;
    std::vector<uint8_t> bytes_;
    size_t n_ = 0;

    static uint64_t mix(uint64_t h) {
        h ^= h >> 32;
        h *= 0xD6E8FEB86659FD93ull;
        h ^= h >> 32;
        return h;
    }
    size_t probe(uint64_t h, const uint8_t *k, size_t n) const {  // slot of k, or the free slot it goes in
        const size_t m = tab_.size() - 1;
        for (size_t i = h & m;; i = (i + 1) & m) {
            const Slot &e = tab_[i];
            if (e.len == kFree) return i;
            if (e.h == h && e.len == n && (n == 0 || std::memcmp(bytes_.data() + e.off, k, n) == 0)) return i;
        }
    }
    void grow(size_t want = 0) {
        std::vector<Slot> old(std::max<size_t>({tab_.size() * 2, want, 1024}), Slot{0, 0, kFree, 0, ~0u, 0});
        old.swap(tab_);
        const size_t m = tab_.size() - 1;
        for (const Slot &e : old)
            if (e.len != kFree) {
                size_t i = e.h & m;
                while (tab_[i].len != kFree) i = (i + 1) & m;
                tab_[i] = e;
            }
    }

  public:
    static uint64_t hash(const uint8_t *k, size_t n) {
        uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
        size_t i = 0;
        for (; i + 8 <= n; i += 8) {
            uint64_t w;
            std::memcpy(&w, k + i, 8);
            h = mix(h ^ w) * 0x9E3779B97F4A7C15ull;
        }
        uint64_t w = 0;
        if (n > i) std::memcpy(&w, k + i, n - i);
        return mix(mix(h ^ w) + n);
    }
    size_t size() const { return n_; }
    // batched lookups: the slot a hash starts probing at, to prefetch ahead of find_hint_h
    const void *slot_addr(uint64_t h) const { return tab_.empty() ? nullptr : &tab_[h & (tab_.size() - 1)]; }
    // find_hint with the hash already computed
    bool find_hint_h(uint64_t h, const uint8_t *k, size_t n, uint32_t *shard, uint32_t *chunk, uint32_t *idx) const {
        if (tab_.empty()) return false;
        const Slot &e = tab_[probe(h, k, n)];
        if (e.len == kFree) return false;
        *shard = e.shard;
        *chunk = e.chunk;
        *idx = e.idx;
        return true;
    }
    // shard of k, or -1
    int64_t find(const uint8_t *k, size_t n) const {
        if (tab_.empty()) return -1;
        const Slot &e = tab_[probe(hash(k, n), k, n)];
        return e.len == kFree ? -1 : (int64_t)e.shard;
    }
    // shard and record hint of k; false when k was never stored
    bool find_hint(const uint8_t *k, size_t n, uint32_t *shard, uint32_t *chunk, uint32_t *idx) const {
        if (tab_.empty()) return false;
        const Slot &e = tab_[probe(hash(k, n), k, n)];
        if (e.len == kFree) return false;
        *shard = e.shard;
        *chunk = e.chunk;
        *idx = e.idx;
        return true;
    }
    // room for `more` keys (of `bytes` key bytes) without rehashing on the way: one table of
    // the final size, not a doubling per step
    void reserve(size_t more, size_t bytes = 0) {
        if ((n_ + more) * 2 > tab_.size()) {
            size_t want = 1024;
            while ((n_ + more) * 2 > want) want <<= 1;
            grow(want);
        }
        if (bytes) bytes_.reserve(bytes_.size() + bytes);
    }
    // the slot a hash starts probing at (prefetch ahead of upsert_h)
    const void *probe_addr(uint64_t h) const { return tab_.empty() ? nullptr : &tab_[h & (tab_.size() - 1)]; }
    // upsert with the hash already computed (KeyMap::hash(k, n))
    int64_t upsert_h(uint64_t h, const uint8_t *k, size_t n, uint32_t shard, uint32_t chunk, uint32_t idx) {
        if ((n_ + 1) * 2 > tab_.size()) grow();
        Slot &e = tab_[probe(h, k, n)];
        if (e.len == kFree) {
            e = Slot{h, bytes_.size(), (uint32_t)n, shard, chunk, idx};
            bytes_.insert(bytes_.end(), k, k + n);
            ++n_;
            return -1;
        }
        const int64_t prev = e.shard;
        e.shard = shard;
        e.chunk = chunk;
        e.idx = idx;
        return prev;
    }
    // put, returning the shard k was stored under before (-1: new key)
    int64_t upsert(const uint8_t *k, size_t n, uint32_t shard, uint32_t chunk, uint32_t idx) {
        if ((n_ + 1) * 2 > tab_.size()) grow();
        const uint64_t h = hash(k, n);
        Slot &e = tab_[probe(h, k, n)];
        if (e.len == kFree) {
            e = Slot{h, bytes_.size(), (uint32_t)n, shard, chunk, idx};
            bytes_.insert(bytes_.end(), k, k + n);
            ++n_;
            return -1;
        }
        const int64_t prev = e.shard;
        e.shard = shard;
        e.chunk = chunk;
        e.idx = idx;
        return prev;
    }
    void put(const uint8_t *k, size_t n, uint32_t shard, uint32_t chunk = ~0u, uint32_t idx = 0) {
        (void)upsert(k, n, shard, chunk, idx);
    }
    void clear() {
        tab_.clear();
        bytes_.clear();
        n_ = 0;
    }
};

// KeyMap split into 16 partitions by key hash: a batch's upserts run one partition per
// host thread, each seeing its keys in record order
class PartKeyMap {
  public:
    static constexpr uint32_t kParts = 16;
    static uint32_t part_of(const uint8_t *k, size_t n) { return (uint32_t)(KeyMap::hash(k, n) >> 60); }
    int64_t find(const uint8_t *k, size_t n) const { return p_[part_of(k, n)].find(k, n); }
    bool find_hint(const uint8_t *k, size_t n, uint32_t *shard, uint32_t *chunk, uint32_t *idx) const {
        return p_[part_of(k, n)].find_hint(k, n, shard, chunk, idx);
    }
    void put(const uint8_t *k, size_t n, uint32_t shard, uint32_t chunk = ~0u, uint32_t idx = 0) {
        p_[part_of(k, n)].put(k, n, shard, chunk, idx);
    }
    KeyMap &part(uint32_t i) { return p_[i]; }
    // batched lookups with the hash computed once (KeyMap::hash(k, n))
    const void *slot_addr(uint64_t h) const { return p_[h >> 60].slot_addr(h); }
    bool find_hint_h(uint64_t h, const uint8_t *k, size_t n, uint32_t *shard, uint32_t *chunk, uint32_t *idx) const {
        return p_[h >> 60].find_hint_h(h, k, n, shard, chunk, idx);
    }
    size_t size() const {
        size_t n = 0;
        for (const auto &m : p_) n += m.size();
        return n;
    }
    void clear() {
        for (auto &m : p_) m.clear();
    }

  private:
    KeyMap p_[kParts];
};

// ---------------------------------------------------------------- phase clock
// host wall time per phase of one call, printed on stderr when `env` is 1
struct PhaseClock {
    bool on = false;
    const char *name;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), t = t0;
    std::string out;
    const char *cur = "setup";
    PhaseClock(const char *nm, const char *env) : name(nm) {
        const char *v = std::getenv(env);
        on = v && *v == '1';
    }
    void mark(const char *next) {  // closes the running phase, starts `next`
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        char b[128];
        snprintf(b, sizeof b, "\n  %8.2f ms  %s", std::chrono::duration<double, std::milli>(now - t).count(), cur);
        out += b;
        t = now;
        cur = next;
    }
    ~PhaseClock() {
        if (!on) return;
        mark("");
        fprintf(stderr, "%s:%s\n  %8.2f ms  total\n", name, out.c_str(),
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};

// ---------------------------------------------------------------- worker pool
// Persistent host workers (created once per process): spawning threads per call cost
// more than a 10k-key lookup batch itself.  run(n, f) calls f(0..n-1) on the workers
// and the caller, and returns when every call has returned.
class WorkerPool {
  public:
    static WorkerPool &get() {
        static WorkerPool pool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1);
        return pool;
    }
    uint32_t size() const { return (uint32_t)workers_.size() + 1; }
    void run(uint32_t ntask, const std::function<void(uint32_t)> &f) {
        std::lock_guard<std::mutex> one(run_mu_);  // one job at a time (callers from several threads)
        std::unique_lock<std::mutex> lk(m_);
        busy_.wait(lk, [&] { return active_ == 0; });  // no worker still holds the last job
        fn_ = &f;
        ntask_ = ntask;
        next_.store(0);
        done_ = 0;
        ++gen_;
        lk.unlock();
        work_.notify_all();
        uint32_t mine = 0;
        for (uint32_t t; (t = next_.fetch_add(1)) < ntask;) {
            f(t);
            ++mine;
        }
        lk.lock();
        done_ += mine;
        // back as soon as every task ran: a worker that woke late finds none left and never
        // calls f (the next run waits for it to leave before it publishes a new job)
        busy_.wait(lk, [&] { return done_ == ntask_; });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            quit_ = true;
        }
        work_.notify_all();
        for (auto &t : workers_) t.join();
    }

  private:
    explicit WorkerPool(uint32_t n) {
        for (uint32_t i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(m_);
            work_.wait(lk, [&] { return quit_ || gen_ != seen; });
            if (quit_) return;
            seen = gen_;
            ++active_;
            const std::function<void(uint32_t)> *f = fn_;
            const uint32_t nt = ntask_;
            lk.unlock();
            uint32_t mine = 0;
            for (uint32_t t; (t = next_.fetch_add(1)) < nt;) {
                (*f)(t);
                ++mine;
            }
            lk.lock();
            done_ += mine;
            --active_;
            busy_.notify_all();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex m_, run_mu_;
    std::condition_variable work_, busy_;
    const std::function<void(uint32_t)> *fn_ = nullptr;
    uint32_t ntask_ = 0, done_ = 0, active_ = 0;
    std::atomic<uint32_t> next_{0};
    uint64_t gen_ = 0;
    bool quit_ = false;
};

// fn(lo, hi) over [0, n) on up to `threads` host threads (inline for small n)
template <class F>
void parallel_ranges(uint32_t n, uint32_t threads, F fn) {
    if (threads <= 1 || n < 2048) {
        fn(0u, n);
        return;
    }
    threads = std::min<uint32_t>({threads, WorkerPool::get().size(), n / 512});
    const uint32_t tasks = threads * 4;  // a few ranges per thread: uneven keys balance out
    const uint32_t per = (n + tasks - 1) / tasks;
    const std::function<void(uint32_t)> job = [&](uint32_t t) {
        const uint32_t lo = t * per, hi = std::min(n, lo + per);
        if (lo < hi) fn(lo, hi);
    };
    WorkerPool::get().run(tasks, job);
}

// out[0] = 0, out[i + 1] = out[i] + val(i) for i < n (uint64), on `threads` host threads: block
// sums, their prefix, then each block's running sum (a million-element prefix was ~2 ms serial)
template <class V>
void parallel_prefix(uint32_t n, uint32_t threads, uint64_t *out, V val) {
    out[0] = 0;
    if (threads <= 1 || n < 65536) {
        for (uint32_t i = 0; i < n; ++i) out[i + 1] = out[i] + val(i);
        return;
    }
    constexpr uint32_t kBlk = 16384;
    const uint32_t nb = (n + kBlk - 1) / kBlk;
    std::vector<uint64_t> bs(nb + 1, 0);
    const std::function<void(uint32_t)> sum = [&](uint32_t b) {
        uint64_t t = 0;
        for (uint32_t i = b * kBlk, e = std::min(n, i + kBlk); i < e; ++i) t += val(i);
        bs[b + 1] = t;
    };
    WorkerPool::get().run(nb, sum);
    for (uint32_t b = 0; b < nb; ++b) bs[b + 1] += bs[b];
    const std::function<void(uint32_t)> put = [&](uint32_t b) {
        uint64_t t = bs[b];
        for (uint32_t i = b * kBlk, e = std::min(n, i + kBlk); i < e; ++i) {
            t += val(i);
            out[i + 1] = t;
        }
    };
    WorkerPool::get().run(nb, put);
}

// ---------------------------------------------------------------- crit-bit index
// Restates CritBitTree.cpp:13-269 over the COMPAT-decoded key prefix of each stored
// record (computed on the GPU at setitem time).  Walk bytes past a key's end read 0
// (as getitem does); crit-bit trees are canonical, so this equals the reference's
// tree whenever the decoded key prefixes equal the true keys.  A tree's leaves are
// records; the caller supplies each leaf's stored key prefix (kp(leaf, &len) -> bytes,
// the escaped key through 251,0) and what a replace or delete does to the leaf (del).
struct Leaf {
    uint32_t chunk, idx;  // global chunk id, slot
};
struct CbtRef {
    int32_t inner = -1;
    Leaf leaf{0, 0};
};
struct CbtInner {
    CbtRef kid[2];
    uint16_t diff_at;
    uint8_t mask;
};
inline int crit_dir(uint8_t mask, uint8_t byte) { return (1 + (mask | byte)) >> 8; }

struct CritBit {
    std::vector<CbtInner> cbt;
    std::vector<int32_t> cbt_free;
    bool has_root = false;
    CbtRef root;

    struct Best {
        int32_t grand = -1, pa = -1;
        int dir = 3;
        Leaf crit{0, 0};
    };
    Best best_match(const std::string &q) const {
        Best b;
        CbtRef p = root;
        while (p.inner >= 0) {
            const CbtInner &n = cbt[(size_t)p.inner];
            uint8_t byte = q.size() > n.diff_at ? (uint8_t)q[n.diff_at] : 0;
            b.dir = crit_dir(n.mask, byte);
            b.grand = b.pa;
            b.pa = p.inner;
            p = n.kid[b.dir];
        }
        b.crit = p.leaf;
        return b;
    }
    // PXSGen_key_eq on a stored key prefix: equal through the key terminator
    static bool key_eq(const uint8_t *crit, uint32_t clen, const std::string &q) {
        bool spec = false;
        for (size_t k = 0; k < clen && k < q.size() && crit[k] == (uint8_t)q[k]; ++k) {
            uint8_t v = crit[k];
            if (!spec && v == kEscByte) {
                spec = true;
            } else if (spec) {
                if (v == kKeyEndByte) return true;
                spec = false;
            }
        }
        return false;
    }

    // CritBitTree::setitem; q = escaped key incl. 251,0.  Returns 0 when inserted, 1 on
    // replace (the old leaf goes to del, the new one takes its place), 2 when the streams
    // part right after a 251 and the reference skips the insert (`if (!spec_mode)
    // insert()`, CritBitTree.cpp:96-100): the record is stored but no walk reaches it.
    template <class KP, class Del>
    int insert(const std::string &q, Leaf nl, KP kp, Del del) {
        CbtRef nref;
        nref.leaf = nl;
        if (!has_root) {
            has_root = true;
            root = nref;
            return 0;
        }
        Best b = best_match(q);
        uint32_t clen;
        const uint8_t *crit = kp(b.crit, &clen);
        size_t k = 0;
        uint16_t diff_at = 0;
        uint8_t crit_rv = 0, src_rv = 0;
        bool spec = false;
        for (;;) {
            if (k >= clen) break;
            crit_rv = crit[k];
            if (k >= q.size()) break;
            src_rv = (uint8_t)q[k];
            ++k;
            if (crit_rv != src_rv) break;
            if (!spec && crit_rv == kEscByte) {
                spec = true;
            } else if (spec) {
                if (crit_rv == kKeyEndByte) {
                    del(b.crit);
                    if (b.pa < 0) root = nref;
                    else cbt[(size_t)b.pa].kid[b.dir] = nref;
                    return 1;
                }
                spec = false;
            }
            ++diff_at;
        }
        if (spec) return 2;
        uint8_t mask = crit_rv ^ src_rv;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask = (uint8_t)((mask & ~(mask >> 1)) ^ 0xff);
        uint8_t at = diff_at < q.size() ? (uint8_t)q[diff_at] : 0;
        int dir = crit_dir(mask, at);
        int32_t in;
        if (!cbt_free.empty()) {
            in = cbt_free.back();
            cbt_free.pop_back();
        } else {
            cbt.emplace_back();
            in = (int32_t)cbt.size() - 1;
        }
        cbt[(size_t)in].diff_at = diff_at;
        cbt[(size_t)in].mask = mask;
        cbt[(size_t)in].kid[dir] = nref;
        int32_t parent = -1;
        int pdir = 0;
        CbtRef p = root;
        while (p.inner >= 0) {
            const CbtInner &n = cbt[(size_t)p.inner];
            if (n.diff_at > diff_at || (n.diff_at == diff_at && n.mask > mask)) break;
            uint8_t byte = q.size() > n.diff_at ? (uint8_t)q[n.diff_at] : 0;
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

    // CritBitTree::getitem's lookup (CritBitTree.cpp:180-196) and contains (:154-178)
    template <class KP>
    bool lookup(const std::string &q, KP kp, Leaf *out) const {
        if (!has_root) return false;
        Best b = best_match(q);
        uint32_t clen;
        const uint8_t *crit = kp(b.crit, &clen);
        if (!key_eq(crit, clen, q)) return false;
        if (out) *out = b.crit;
        return true;
    }

    // CritBitTree::delitem (CritBitTree.cpp:107-152): 0 deleted (the leaf goes to del), 1 absent
    template <class KP, class Del>
    int remove(const std::string &q, KP kp, Del del) {
        if (!has_root) return 1;
        Best b = best_match(q);
        uint32_t clen;
        const uint8_t *crit = kp(b.crit, &clen);
        if (!key_eq(crit, clen, q)) return 1;
        if (b.pa < 0) {
            has_root = false;
            root = CbtRef{};
        } else {
            const CbtRef other = cbt[(size_t)b.pa].kid[1 - b.dir];
            if (b.grand < 0) {
                root = other;
            } else {
                CbtInner &g = cbt[(size_t)b.grand];
                int gd = (g.kid[0].inner == b.pa) ? 0 : 1;
                g.kid[gd] = other;
            }
            cbt_free.push_back(b.pa);
        }
        del(b.crit);
        return 0;
    }

    // CritBitTree::iter (CBTGHelper / CBTGen, CritBitTree.h:55-157): follow the prefix's
    // crit bits; from the first node whose diff_at is past the prefix take the whole
    // subtree (kid 0 first).  The first leaf reached must start with the prefix
    // (startswith(leaf)), else the generator yields NULL and stops; later leaves are
    // unchecked.  Returns false for an empty tree.
    template <class Starts>
    bool iter(const std::string &p, Starts startswith, std::vector<Leaf> &out) const {
        if (!has_root) return false;
        bool harvest = false;
        std::vector<std::pair<CbtRef, bool>> stack{{root, false}};
        while (!stack.empty()) {
            auto [ref, include_all] = stack.back();
            stack.pop_back();
            if (ref.inner < 0) {
                if (!harvest && !startswith(ref.leaf)) break;
                harvest = true;
                out.push_back(ref.leaf);
                continue;
            }
            const CbtInner &n = cbt[(size_t)ref.inner];
            uint8_t crit = p.size() > n.diff_at ? (uint8_t)p[n.diff_at] : 0;
            int direct = crit_dir(n.mask, crit);
            if (!include_all && n.diff_at >= p.size()) include_all = true;
            if (include_all) {
                stack.push_back({n.kid[1], true});
                stack.push_back({n.kid[0], true});
            } else {
                stack.push_back({n.kid[direct], false});
            }
        }
        return true;
    }
    void clear() {
        cbt.clear();
        cbt_free.clear();
        has_root = false;
        root = CbtRef{};
    }
};

}  // namespace pxh
