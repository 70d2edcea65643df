/* oracle/pxo.h — TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of the PiXiu hot path (escape, Ukkonen GST +
 * stream encoder with exact pool accounting, PXSGen-compatible decoder, exact
 * decoder).  Used only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the CHECKER; the product (pixiu_amd/) never links it.
 *
 * Parity pinning: validated against the reference itself (oracle/_ref, built
 * from /root/reference/src by oracle/Makefile) by tests/test_oracle_vs_ref.py,
 * and against the committed golden vectors in tests/golden/.
 *
 * Every handle is independent (no globals), unlike the reference.
 */
#ifndef PXO_H
#define PXO_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct pxo_shard pxo_shard;

/* decode modes */
#define PXO_COMPAT 0 /* byte-exact with the reference PXSGen (PiXiuStr.h:129-198) */
#define PXO_EXACT 1  /* correct LZ expansion (overlap test on the absolute cursor) */

/* error codes (negative) */
#define PXO_EINVAL -1  /* empty key, oversize doc (> 65535 escaped bytes) */
#define PXO_ESPACE -2  /* caller buffer too small */
#define PXO_ECORRUPT -3 /* malformed compressed bytes / reference would dereference NULL */
#define PXO_EHANG -4   /* the reference decoder would loop forever (empty periodic source) */

pxo_shard *pxo_new(void);
void pxo_free(pxo_shard *s);

/* PiXiuCtrl::setitem (PiXiuCtrl.cpp:12-47) for one record. Returns 0 or 1 (replaced a
 * duplicate key), or a negative error.  Reports chunk number and chunk-local slot. */
int pxo_set(pxo_shard *s, const uint8_t *k, int klen, const uint8_t *v, int vlen,
            uint32_t *chunk_no, uint32_t *idx);

/* compressed bytes of (chunk, idx) */
int pxo_comp(pxo_shard *s, uint32_t chunk, uint32_t idx, uint8_t *out, int cap);

/* PiXiuStr::parse(from,to) on (chunk, idx) in the given mode. */
int pxo_parse(pxo_shard *s, uint32_t chunk, uint32_t idx, int from, int to, int mode,
              uint8_t *out, int cap);

/* PiXiuCtrl::getitem (PiXiuCtrl.cpp:59-61) drained; -5 == NULL (missing key) */
#define PXO_NOTFOUND -5
int pxo_get(pxo_shard *s, const uint8_t *k, int klen, int mode, uint8_t *out, int cap);

/* where the key's record lives (chunk number, slot); PXO_NOTFOUND if absent */
int pxo_locate(pxo_shard *s, const uint8_t *k, int klen, uint32_t *chunk, uint32_t *idx);

/* PiXiuCtrl::contains (1/0) and ::delitem (0 deleted, 1 not found) */
int pxo_contains(pxo_shard *s, const uint8_t *k, int klen);
/* PiXiuCtrl::reinsert on closed chunk c (PiXiuCtrl.cpp:88-114) */
int pxo_reinsert(pxo_shard *s, uint32_t c);
int pxo_delete(pxo_shard *s, const uint8_t *k, int klen);
/* PiXiuCtrl::iter: (chunk, idx) of the yielded records in order; count, PXO_NOTFOUND
   for an empty tree, PXO_ESPACE if cap is too small. */
int pxo_iter(pxo_shard *s, const uint8_t *prefix, int plen, uint32_t *chunk_out, uint32_t *idx_out, int cap);

uint32_t pxo_num_chunks(pxo_shard *s);
uint32_t pxo_chunk_records(pxo_shard *s, uint32_t chunk);
/* pool counters of the live GST (MemPool.h:14-22: nth, used_num) */
void pxo_pool_state(pxo_shard *s, int *pools, int *used_blocks);
int pxo_pool_trace(int n, const uint8_t *docs, const uint64_t *doc_off, uint32_t *chunk_no, int32_t *pools,
                   int32_t *used);

/* PiXiuStr_init / PiXiuStr_init_key (PiXiuStr.cpp:8-14, 228-271) */
int pxo_escape(const uint8_t *src, int n, int is_key, uint8_t *out, int cap);

/* raw stream encoder (PiXiuStr.cpp:16-118): cmd >= 0 compress(idx=cmd,pos), -3 pass */
int pxo_stream(int n, const int *cmd, const int *pos, const uint8_t *val, uint8_t *out, int cap);

/* Whole-shard driver with the same layout as refx_run (oracle/ref_driver.cpp):
 * inserts records [0,n) in order into a fresh shard, then (if do_get) getitem()s
 * every key in `mode`.  comp_off / dec_off have n+1 entries. */
int pxo_run(int n, const uint8_t *keys, const uint64_t *koff, const uint32_t *klen,
            const uint8_t *vals, const uint64_t *voff, const uint32_t *vlen,
            uint8_t *comp, uint64_t comp_cap, uint64_t *comp_off,
            uint32_t *chunk_no, uint32_t *idx,
            int do_get, int mode, uint8_t *dec, uint64_t dec_cap, uint64_t *dec_off);

/* Same as pxo_run but docs are already escaped/assembled (CSR), no CritBit:
 * the per-shard encoder only.  Used as the GPU-parity checker at full sizes. */
int pxo_encode_docs(int n, const uint8_t *docs, const uint64_t *doc_off,
                    uint8_t *comp, uint64_t comp_cap, uint64_t *comp_off,
                    uint32_t *chunk_no, uint32_t *idx);

/* decode (idx, from, to) against a caller-supplied chunk of n compressed records */
int pxo_decode_chunk(int n, const uint8_t *comp, const uint64_t *off, int idx, int from, int to, int mode,
                     uint8_t *out, int cap);

#ifdef __cplusplus
}
#endif
#endif
