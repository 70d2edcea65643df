/* pixiu_amd.h — C ABI of the MI355X-native PiXiu batch compress/query core.
 *
 * This is the drop-in boundary.  Every entry point is plain C:
 * pointers, sizes and status codes; no C++ or torch types cross it.  The
 * source-compatible C++ facade (include/PiXiuCtrl.h) and the Python binding
 * (pixiu_amd/__init__.py) are thin layers over these calls.
 *
 * Object model: a px_ctx is a sharded store.  Records are assigned, in arrival
 * order, to shards of `records_per_shard` records; every shard is an independent
 * PiXiuCtrl-equivalent (own generalized suffix tree, chunks, CritBit index), so
 * shard s's compressed bytes equal what the reference produces when fed exactly
 * shard s's records.  records_per_shard == 0 means ONE shard: the exact
 * single-instance semantics of the reference PiXiuCtrl.
 *
 * Reference interfaces replaced (file:line in Thunderchen/PiXiu src/):
 *   px_open / px_close ........ PiXiuCtrl::init_prop / free_prop   (PiXiuCtrl.cpp:77-86)
 *   px_set_batch .............. PiXiuCtrl::setitem                  (PiXiuCtrl.cpp:12-47)
 *   px_set_docs ............... PiXiuCtrl::setitem(k, 0, NULL, 0, reinsert)  (PiXiuCtrl.cpp:26-40, ready docs)
 *   px_flush .................. (none: the write-behind queue of one-record setitem calls)
 *   px_get_batch .............. PiXiuCtrl::getitem + PXSGen drain   (PiXiuCtrl.cpp:59-61, PiXiuStr.h:129-198)
 *   px_get_batch_dev .......... the same, keys and results in device memory
 *   px_contains_batch ......... PiXiuCtrl::contains                 (PiXiuCtrl.cpp:55-57)
 *   px_del_batch .............. PiXiuCtrl::delitem                  (PiXiuCtrl.cpp:63-69)
 *   px_iter ................... PiXiuCtrl::iter -> CBTGen           (PiXiuCtrl.cpp:71-75, CritBitTree.h:55-157)
 *   px_parse_batch ............ PiXiuStr::parse(from,to,chunk)      (PiXiuStr.cpp:166-176)
 *   px_export ................. cbt_chunk->getitem(idx) bytes       (PiXiuStr.cpp:202-206, main.cpp:67)
 *   px_locate_batch ........... CritBitTree::getitem's lookup       (CritBitTree.cpp:180-196, before the parse)
 *   px_reinsert ............... PiXiuCtrl::reinsert(PiXiuChunk *&)  (PiXiuCtrl.cpp:88-114)
 *   px_save / px_load ......... (none: the reference has no persistence; chunk blob v1)
 *
 * All calls are synchronous on the context's HIP stream.  A context is not
 * thread-safe; distinct contexts are fully independent (no globals).
 */
#ifndef PIXIU_AMD_H
#define PIXIU_AMD_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef enum px_status {
    PX_OK = 0,
    PX_EINVAL = 1,      /* bad argument, empty key, escaped doc > 65,535 B */
    PX_ECAPACITY = 2,   /* internal arena sizing failure */
    PX_EREFCRASH = 3,   /* input on which the reference dereferences NULL (its GST bug) */
    PX_ECORRUPT = 4,    /* malformed compressed bytes */
    PX_EHANG = 5,       /* input on which the reference decoder never terminates */
    PX_EDEPTH = 6,      /* decode nesting deeper than opts.decode_depth */
    PX_ESPACE = 7,      /* output buffer too small */
    PX_ENOTFOUND = 8,   /* getitem/contains/delitem of a missing key */
    PX_EHIP = 9,        /* HIP runtime error */
    PX_ENOMEM = 10      /* device allocation failed */
} px_status;

typedef enum px_mode {
    PX_COMPAT = 0, /* byte-exact with the reference PXSGen, bugs included */
    PX_EXACT = 1   /* correct LZ expansion: equals the original escaped doc, except in a record
                      holding a small reference token of length 251 (the reference encoder writes
                      its length byte as 251, which every decoder reads as an escape pair:
                      PiXiuStr.cpp:61-78) -- those bytes are lost at setitem, in the reference
                      too, and such a record's exact expansion is shorter than its doc */
} px_mode;

typedef struct px_opts {
    int device;                 /* HIP device ordinal */
    uint32_t records_per_shard; /* 0 = single shard (reference semantics) */
    uint32_t decode_depth;      /* frames per decode stack; 0 = 4096 */
    uint32_t decode_waves;      /* concurrent decode wavefronts; 0 = one per query, up to 16,384 */
    uint32_t host_threads;      /* host threads for batch key lookups; 0 = min(16, cores) */
    uint32_t defer_bytes;       /* write-behind of host px_set_batch calls (records_per_shard == 0
                                   only): records are queued and stored together once this many
                                   raw bytes are pending, or by px_flush / any other call on the
                                   context; 0 = off (every call stores at once).  See px_flush. */
    uint32_t retain_mb;         /* device memory the heap keeps cached in wholly free slabs after a
                                   set batch (the rest goes back to the driver); 0 = what that
                                   batch needed at its peak beyond what stays live (similar
                                   batches then never re-allocate), capped at half of the device
                                   memory free to the process (free + cached); 0xffffffff = keep
                                   everything.
                                   px_trim returns cached memory on request. */
} px_opts;

typedef struct px_ctx px_ctx;

/* per-record result of px_set_batch */
typedef struct px_set_result {
    uint32_t status;   /* px_status */
    uint32_t replaced; /* 1 = CBT_SET_REPLACE (duplicate key in the same shard) */
    uint32_t shard;
    uint32_t chunk;    /* chunk sequence number inside the shard (rotation count); PX_PENDING
                          while a deferred record waits in the write-behind queue */
    uint32_t idx;      /* chunk-local slot (the `idx` that references point at); PX_PENDING */
    uint32_t comp_len; /* compressed length; PX_PENDING */
    uint32_t doc_len;  /* escaped doc length (esc(k)+[251,0]+esc(v)+[251,2]) */
    uint32_t pad;
} px_set_result;

#define PX_PENDING 0xffffffffu /* px_set_result field of a record still in the write-behind queue */

/* a stored record, as addressed by px_parse_batch / px_export */
typedef struct px_rec {
    uint32_t shard, chunk, idx;
    int32_t from, to; /* parse range (escaped coordinates); [0, 65535) = whole record */
} px_rec;

typedef struct px_stats {
    uint64_t records, shards, chunks;
    uint64_t raw_bytes, doc_bytes, comp_bytes;
    uint64_t ub_reads;        /* reads the reference makes out of bounds (UB there) */
    uint64_t device_bytes;    /* device memory held now: the heap (live + cached free) plus the
                                 mapped record-store arena */
    double last_set_stage_ms;     /* GPU events around the encode stage and k_gst_emit of the last
                                     px_set_batch (= last_encode_stage_ms + last_emit_kernel_ms) */
    double last_decode_kernel_ms; /* the getitem stage of the last get/parse batch: k_gather + k_decode
                                     (GPU events around both launches) */
    double last_encode_stage_ms;  /* the encode stage alone -- the text -> encoder-message pass: the
                                     suffix-array pipeline (px_psa.hip, incl. its host-driven steps)
                                     for suffix-array shards and k_gst_encode for walked ones, GPU
                                     events from before the first to after the last of its kernels.
                                     bench.py's roofline.achieved divides by this */
    double last_emit_kernel_ms;   /* k_gst_emit (stream encoder -> compressed bytes) alone */
    double last_get_lookup_ms;    /* host key -> record lookups of the last px_get_batch */
    double last_get_call_ms;      /* wall time inside the last px_get_batch call */
    double last_psa_ms;           /* the suffix-array pass of the last px_set_batch (host wall) */
    uint64_t last_psa_shards;     /* shards the last px_set_batch encoded by the suffix-array pass */
    uint64_t last_walk_shards;    /* shards it walked with k_gst_encode */
    double last_psa_sort_ms;      /* suffix-array pass: text gather + suffix sorting (GPU events) */
    double last_psa_lcp_ms;       /*   nearest-smaller-position links + their lcp values */
    double last_psa_msg_ms;       /*   messages, earliest occurrences, placement */
    uint64_t last_psa_iters;      /*   prefix-doubling steps after the first sort */
    uint64_t span_entries;        /* span-table entries held (8 bytes each) */
    uint64_t last_gather_queries; /* queries of the last get/parse batch served by k_gather */
    double last_span_build_ms;    /* span-table build of the last px_set_batch (host wall) */
    uint64_t last_psa_rounds;     /* suffix-array rounds of the last px_set_batch (one per chunk window) */
    uint64_t last_psa_rotations;  /* chunk rotations the suffix-array path found in it (MemPool emulation) */
    double last_psa_pool_ms;      /* MemPool emulation: leaves, split candidates, pool scan (GPU events) */
    uint64_t device_live_bytes;   /* device memory in use by stored data (records, indexes, arenas) */
    uint64_t device_peak_bytes;   /* the most the heap has held (set-batch scratch at its peak) */
    uint64_t deferred_records;    /* records that went through the write-behind queue */
    uint64_t deferred_flushes;    /* write-behind flushes (each one px_set_batch of the queue) */
    uint64_t deferred_mismatch;   /* deferred records whose `replaced`, returned at call time, differed
                                     from the stored result (only possible when a queued record's
                                     compat-decoded key is not its key: reported, never hidden) */
    uint64_t last_get_device_keys; /* keys of the last px_get_batch resolved by the device key index
                                     (0: the batch resolved its keys on the host) */
    uint64_t last_set_peak_bytes;  /* device memory in use at the peak of the last px_set_batch
                                     (heap live bytes incl. scratch, plus the mapped store arena) */
    /* device memory held for stored data, by structure (allocated bytes; DESIGN.md §2 has the
       per-record and per-text-byte table).  Their sum is device_live_bytes less small control
       blocks and the write-behind queue. */
    uint64_t mem_text_bytes;    /* suffix-array shards' live-chunk text (the next batch sorts it) */
    uint64_t mem_tree_bytes;    /* walked shards' arenas: nodes, child hash, live-chunk text */
    uint64_t mem_comp_bytes;    /* compressed records (8-byte aligned) */
    uint64_t mem_lane_bytes;    /* lane-walk entries, 16 B per segment */
    uint64_t mem_seg_bytes;     /* segment index, 16 B per segment */
    uint64_t mem_pidx_bytes;    /* position index, 2 B per 16 doc bytes */
    uint64_t mem_span_bytes;    /* span tables (8 B per span) and their tile index (4 B per 32 B out) */
    uint64_t mem_slot_bytes;    /* chunk slot tables (48 B per slot of capacity) */
    uint64_t mem_keyidx_bytes;  /* device key index: records (80 B), raw keys, hash slots (16 B) */
} px_stats;

px_ctx *px_open(const px_opts *opts);
void px_close(px_ctx *ctx);
const char *px_strerror(int status);

/* Batch setitem.  Record i: key = keys[koff[i] .. koff[i+1]), value =
 * vals[voff[i] .. voff[i+1]) (empty value = key-only record).  If on_device, the
 * four pointers are device pointers (inputs already resident in HBM); otherwise
 * host pointers.  res (host, n entries) may be NULL.  Returns PX_OK if every
 * record was stored, else the first failing status (others may have succeeded). */
int px_set_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff,
                 const uint8_t *vals, const uint64_t *voff, int on_device, px_set_result *res);

/* Ready docs (PiXiuCtrl::setitem(k, 0, NULL, 0, reinsert), PiXiuCtrl.cpp:26-40): record i
 * is the escaped doc docs[doff[i] .. doff[i+1]) as PiXiuStr::data holds it, stored without
 * escaping; its CritBit key is its prefix through the first 251,0.  reinsert != 0 skips
 * the Glob_Reinsert_Chunk trigger (PiXiuCtrl.cpp:26-29), as the reference's flag does. */
int px_set_docs(px_ctx *ctx, uint32_t n, const uint8_t *docs, const uint64_t *doff, int on_device, int reinsert,
                px_set_result *res);

/* Store every record of the write-behind queue (opts.defer_bytes).  A deferred px_set_batch
 * returns at once: status PX_OK (or PX_EINVAL for an invalid record, which is not queued),
 * `replaced` resolved at call time from the CritBit of the stored records and the queued
 * keys (a key equal to a queued one flushes the queue first), doc_len, and PX_PENDING for
 * chunk / idx / comp_len.  Every other call on the context flushes first, so reads always
 * see every record set before them; px_reset / px_close drop the queue.  Chunk rotation
 * depends only on the doc order, so the stored bytes equal those of one call per record.
 * last (may be NULL): the result of the most recently stored record.  Returns PX_OK, or
 * the first failing status among the records stored since the previous px_flush. */
int px_flush(px_ctx *ctx, px_set_result *last);

/* Batch getitem: keys are host CSR.  The expanded doc of key i lands in
 * out[out_off[i] .. out_off[i] + out_len[i]) (out is a device pointer when
 * out_on_device, else host).  status[i] = PX_OK or PX_ENOTFOUND/...  If out_cap
 * is too small the call returns PX_ESPACE and *needed (if non-NULL) holds the
 * required capacity.  out_off/out_len/status are host arrays of n entries. */
int px_get_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, int mode,
                 uint8_t *out, uint64_t out_cap, int out_on_device, uint64_t *out_off,
                 uint32_t *out_len, uint32_t *status, uint64_t *needed);

/* Batch getitem with everything in device memory: keys + koff[n + 1] (CSR offsets into
 * keys), out, out_off / out_len / status (n entries each) are device pointers; the results are
 * written on the device and complete when the call returns.  Same results and return codes as
 * px_get_batch, except that when out_cap is too small only *needed is defined (with
 * PX_ESPACE).  Keys the device key index does not answer go the host path (keys copied down,
 * results up).  The keys are read in place and never past keys + koff[n]: no padding is
 * needed after the last key (its tail is read byte by byte). */
int px_get_batch_dev(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, int mode,
                     uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint32_t *out_len,
                     uint32_t *status, uint64_t *needed);

/* Batch PiXiuStr::parse(from, to) of stored records (the kernel-level boundary). */
int px_parse_batch(px_ctx *ctx, uint32_t n, const px_rec *recs, int mode, uint8_t *out,
                   uint64_t out_cap, int out_on_device, uint64_t *out_off, uint32_t *out_len,
                   uint32_t *status, uint64_t *needed);

/* contains / delitem by key (host keys).  result[i] = 1/0 (contains) or
 * 0 deleted / 1 CBT_DEL_NOT_FOUND (delitem), as the reference returns. */
int px_contains_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff,
                      uint32_t *result);
int px_del_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff,
                 uint32_t *result);

/* PiXiuCtrl::iter(prefix) (PiXiuCtrl.cpp:71-75; CBTGen/CBTGHelper, CritBitTree.h:55-157):
 * the records the reference's generator yields, in yield order (crit-bit order under
 * the escaped prefix; nothing when the first record reached does not start with it).
 * Expand them with px_parse_batch over [0, 65535).  Shards are visited in id order
 * (records_per_shard = 0 is the reference's single tree).  PX_ENOTFOUND: every tree is
 * empty (the reference returns a NULL generator).  PX_ESPACE: *n_out = records needed. */
int px_iter(px_ctx *ctx, const uint8_t *prefix, uint64_t prefix_len, px_rec *recs, uint32_t cap,
            uint32_t *n_out);

/* The lookup half of getitem (CritBitTree.cpp:180-196): the record each key resolves to,
 * recs[i] = {shard, chunk, idx, 0, 65535}, status[i] = PX_OK or PX_ENOTFOUND.  A caller
 * expands it later with px_parse_batch (a lazily drained PXSGen). */
int px_locate_batch(px_ctx *ctx, uint32_t n, const uint8_t *keys, const uint64_t *koff, px_rec *recs,
                    uint32_t *status);

/* PiXiuCtrl::reinsert(PiXiuChunk *&) called directly (PiXiuCtrl.cpp:88-114): chunk `chunk`
 * (sequence number) of shard `shard` is compacted -- every live record, compat-expanded,
 * is set again as a ready doc (rotation trigger only) and the chunk's records are gone.
 * Defined for a closed slot-full chunk: the reference visits all 65,535 slots and
 * dereferences NULL otherwise.  PX_EINVAL for the live chunk, a chunk with empty slots,
 * one with no live record left (compacted already), or an unknown one. */
int px_reinsert(px_ctx *ctx, uint32_t shard, uint32_t chunk);

/* Compressed bytes of stored records, copied to host CSR (out_off has n+1 entries). */
int px_export(px_ctx *ctx, uint32_t n, const px_rec *recs, uint8_t *out, uint64_t out_cap,
              uint64_t *out_off);

int px_stats_get(px_ctx *ctx, px_stats *st);

/* The packed compressed bytes of the last px_set_batch (records in batch order, each
 * padded to 8 B): the blob multi-GPU runs gather to rank 0 over RCCL.  dst may be
 * NULL to query *bytes. */
int px_last_store(px_ctx *ctx, uint8_t *dst, uint64_t cap, int dst_on_device, uint64_t *bytes);

/* Import n compressed records (host CSR: comp[off[i] .. off[i+1])) as one chunk of a
 * new read-only shard (chunk 0, slots 0..n-1), e.g. records exported by px_export.
 * They can then be expanded with px_parse_batch. */
int px_import_chunk(px_ctx *ctx, uint32_t n, const uint8_t *comp, const uint64_t *off, uint32_t *shard);

/* Chunk blob: the wire / on-disk format of stored records (v1; SURVEY.md §8f row 3 --
 * the reference keeps everything in memory and has no such format).  Little-endian:
 *   header  64 B : u32 magic "PXCB" (0x42435850), u32 version (1), u32 n_chunks,
 *                  u32 n_records, u64 data_off, u64 data_bytes, u32 flags, 28 B zero
 *   chunks  16 B : u32 shard (source shard id), u32 chunk (sequence in that shard),
 *                  u32 first (index of its first record), u32 n (records, <= 65,535)
 *   records 16 B : u64 off (into data), u32 comp_len, u32 doc_len | 1 << 31 (dead)
 *   data         : every record's compressed bytes (8-byte aligned), at data_off
 * Record i of a chunk is the chunk-local slot `idx` that references point at, so a
 * chunk's records decode on their own (no cross-chunk references).
 *
 * px_save writes every chunk of the context (dst NULL: *bytes = size needed;
 * PX_ESPACE if cap is short).  px_load adds a blob's chunks as read-only chunks and
 * indexes their live records (CritBit over the decoded key prefixes): getitem,
 * contains, iter and delitem then work on them.  Each source shard becomes a new
 * shard (*first_shard = the first one); a records_per_shard = 0 context must be
 * empty and takes every chunk into its single shard.  Records set after a load start
 * a fresh chunk (the suffix tree of a loaded chunk is not rebuilt). */
int px_save(px_ctx *ctx, uint8_t *dst, uint64_t cap, int dst_on_device, uint64_t *bytes);
int px_load(px_ctx *ctx, const uint8_t *src, uint64_t len, int src_on_device, uint32_t *first_shard);

/* Drop every stored record (PiXiuCtrl::free_prop + init_prop, PiXiuCtrl.cpp:77-86) while
 * keeping the context's device memory for reuse. */
int px_reset(px_ctx *ctx);

/* Give cached free device memory back to the driver until at most keep_bytes stay cached
 * (wholly free 1 GiB heap slabs; live data is never moved). */
int px_trim(px_ctx *ctx, uint64_t keep_bytes);

/* HIP stream the context runs on (a hipStream_t), for callers that order their
 * own work against it. */
void *px_stream(px_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif
