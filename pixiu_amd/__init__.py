"""pixiu_amd — MI355X-native batch compress/query core for PiXiu.

Python binding over the C ABI in ``include/pixiu_amd.h`` (ctypes; no torch types
cross the boundary).  The compute path is the HIP library ``libpixiu_amd.so``
built in-tree by ``__graft_entry__.build()``; there is no CPU fallback: importing
this package without the library, or opening a store without a GPU, raises.

    from pixiu_amd import Store
    st = Store(records_per_shard=64)
    st.set_batch(keys, values)            # PiXiuCtrl::setitem, batched
    docs = st.get_batch(keys)             # PiXiuCtrl::getitem + PXSGen drain (compat)
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

__all__ = ["Store", "PxError", "COMPAT", "EXACT", "lib_path", "load_library", "STATUS"]

COMPAT = 0
EXACT = 1

STATUS = {
    0: "PX_OK", 1: "PX_EINVAL", 2: "PX_ECAPACITY", 3: "PX_EREFCRASH", 4: "PX_ECORRUPT",
    5: "PX_EHANG", 6: "PX_EDEPTH", 7: "PX_ESPACE", 8: "PX_ENOTFOUND", 9: "PX_EHIP", 10: "PX_ENOMEM",
}
PX_OK, PX_EINVAL, PX_ESPACE, PX_ENOTFOUND, PX_EHIP, PX_ENOMEM = 0, 1, 7, 8, 9, 10
PX_PENDING = 0xFFFFFFFF  # px_set_result chunk / idx / comp_len of a record in the write-behind queue

_HERE = os.path.dirname(os.path.abspath(__file__))


def lib_path() -> str:
    # PIXIU_AMD_LIB selects a debug build (e.g. libpixiu_amd_trace.so) for tools/
    return os.environ.get("PIXIU_AMD_LIB") or os.path.join(_HERE, "libpixiu_amd.so")


class PxError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        super().__init__(f"{what}: {STATUS.get(code, code)}")
        self.code = code


class PxOpts(C.Structure):
    _fields_ = [("device", C.c_int), ("records_per_shard", C.c_uint32), ("decode_depth", C.c_uint32),
                ("decode_waves", C.c_uint32), ("host_threads", C.c_uint32), ("defer_bytes", C.c_uint32),
                ("retain_mb", C.c_uint32)]


class PxSetResult(C.Structure):
    _fields_ = [("status", C.c_uint32), ("replaced", C.c_uint32), ("shard", C.c_uint32),
                ("chunk", C.c_uint32), ("idx", C.c_uint32), ("comp_len", C.c_uint32),
                ("doc_len", C.c_uint32), ("pad", C.c_uint32)]


class PxRec(C.Structure):
    _fields_ = [("shard", C.c_uint32), ("chunk", C.c_uint32), ("idx", C.c_uint32),
                ("from_", C.c_int32), ("to", C.c_int32)]


class PxStats(C.Structure):
    _fields_ = [("records", C.c_uint64), ("shards", C.c_uint64), ("chunks", C.c_uint64),
                ("raw_bytes", C.c_uint64), ("doc_bytes", C.c_uint64), ("comp_bytes", C.c_uint64),
                ("ub_reads", C.c_uint64), ("device_bytes", C.c_uint64),
                ("last_set_stage_ms", C.c_double), ("last_decode_kernel_ms", C.c_double),
                ("last_encode_stage_ms", C.c_double), ("last_emit_kernel_ms", C.c_double),
                ("last_get_lookup_ms", C.c_double), ("last_get_call_ms", C.c_double),
                ("last_psa_ms", C.c_double), ("last_psa_shards", C.c_uint64), ("last_walk_shards", C.c_uint64),
                ("last_psa_sort_ms", C.c_double), ("last_psa_lcp_ms", C.c_double), ("last_psa_msg_ms", C.c_double),
                ("last_psa_iters", C.c_uint64), ("span_entries", C.c_uint64), ("last_gather_queries", C.c_uint64),
                ("last_span_build_ms", C.c_double), ("last_psa_rounds", C.c_uint64),
                ("last_psa_rotations", C.c_uint64), ("last_psa_pool_ms", C.c_double),
                ("device_live_bytes", C.c_uint64), ("device_peak_bytes", C.c_uint64),
                ("deferred_records", C.c_uint64), ("deferred_flushes", C.c_uint64),
                ("deferred_mismatch", C.c_uint64), ("last_get_device_keys", C.c_uint64),
                ("last_set_peak_bytes", C.c_uint64),
                ("mem_text_bytes", C.c_uint64), ("mem_tree_bytes", C.c_uint64), ("mem_comp_bytes", C.c_uint64),
                ("mem_lane_bytes", C.c_uint64), ("mem_seg_bytes", C.c_uint64), ("mem_pidx_bytes", C.c_uint64),
                ("mem_span_bytes", C.c_uint64), ("mem_slot_bytes", C.c_uint64), ("mem_keyidx_bytes", C.c_uint64)]


SET_RESULT_DTYPE = np.dtype([("status", "<u4"), ("replaced", "<u4"), ("shard", "<u4"), ("chunk", "<u4"),
                             ("idx", "<u4"), ("comp_len", "<u4"), ("doc_len", "<u4"), ("pad", "<u4")])
REC_DTYPE = np.dtype([("shard", "<u4"), ("chunk", "<u4"), ("idx", "<u4"), ("from", "<i4"), ("to", "<i4")])

# every symbol include/pixiu_amd.h declares
EXPORTS = ["px_open", "px_close", "px_strerror", "px_set_batch", "px_get_batch", "px_parse_batch",
           "px_contains_batch", "px_del_batch", "px_export", "px_stats_get", "px_stream", "px_reset",
           "px_last_store", "px_import_chunk", "px_iter", "px_save", "px_load", "px_locate_batch", "px_reinsert",
           "px_set_docs", "px_flush", "px_trim", "px_get_batch_dev"]

_LIB = None


def load_library() -> C.CDLL:
    """Load the in-tree HIP library; raises loudly when it is missing (no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise ImportError(f"pixiu_amd: HIP library {path} is missing; run __graft_entry__.build()")
    lib = C.CDLL(path)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    lib.px_open.restype = vp
    lib.px_open.argtypes = [C.POINTER(PxOpts)]
    lib.px_close.argtypes = [vp]
    lib.px_strerror.restype = C.c_char_p
    lib.px_strerror.argtypes = [i32]
    lib.px_set_batch.argtypes = [vp, u32, vp, vp, vp, vp, i32, vp]
    lib.px_get_batch.argtypes = [vp, u32, vp, vp, i32, vp, u64, i32, vp, vp, vp, vp]
    lib.px_get_batch_dev.argtypes = [vp, u32, vp, vp, i32, vp, u64, vp, vp, vp, vp]
    lib.px_parse_batch.argtypes = [vp, u32, vp, i32, vp, u64, i32, vp, vp, vp, vp]
    lib.px_contains_batch.argtypes = [vp, u32, vp, vp, vp]
    lib.px_del_batch.argtypes = [vp, u32, vp, vp, vp]
    lib.px_export.argtypes = [vp, u32, vp, vp, u64, vp]
    lib.px_stats_get.argtypes = [vp, C.POINTER(PxStats)]
    lib.px_stream.restype = vp
    lib.px_stream.argtypes = [vp]
    lib.px_reset.argtypes = [vp]
    lib.px_last_store.argtypes = [vp, vp, u64, i32, vp]
    lib.px_import_chunk.argtypes = [vp, u32, vp, vp, vp]
    lib.px_iter.argtypes = [vp, vp, u64, vp, u32, vp]
    lib.px_save.argtypes = [vp, vp, u64, i32, vp]
    lib.px_load.argtypes = [vp, vp, u64, i32, vp]
    lib.px_locate_batch.argtypes = [vp, u32, vp, vp, vp, vp]
    lib.px_reinsert.argtypes = [vp, u32, u32]
    lib.px_set_docs.argtypes = [vp, u32, vp, vp, i32, i32, vp]
    lib.px_flush.argtypes = [vp, vp]
    lib.px_trim.argtypes = [vp, u64]
    _LIB = lib
    return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def csr(items) -> tuple:
    """list of bytes -> (uint8 buffer, uint64 offsets[n+1])"""
    lens = np.fromiter((len(x) for x in items), dtype=np.uint64, count=len(items))
    off = np.zeros(len(items) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    buf = np.frombuffer(b"".join(items), np.uint8).copy() if len(items) else np.zeros(0, np.uint8)
    if buf.size == 0:
        buf = np.zeros(1, np.uint8)
    return buf, off


class Store:
    """A sharded PiXiu store on one GPU (px_ctx).  records_per_shard=0: one shard,
    i.e. exactly the reference's single PiXiuCtrl instance."""

    def __init__(self, records_per_shard: int = 0, device: int = 0, decode_depth: int = 0,
                 decode_waves: int = 0, host_threads: int = 0, defer_bytes: int = 0, retain_mb: int = 0):
        """defer_bytes > 0 (records_per_shard == 0 only): host set_batch calls go through the
        write-behind queue (px_flush); retain_mb: cached free device memory kept after a set
        batch (0: what the batch needed at its peak, 0xFFFFFFFF: all; see trim())."""
        self._lib = load_library()
        opts = PxOpts(device, records_per_shard, decode_depth, decode_waves, host_threads, defer_bytes, retain_mb)
        h = self._lib.px_open(C.byref(opts))
        if not h:
            raise PxError(9, "px_open (no usable HIP device?)")
        self._h = C.c_void_p(h)
        self._need = np.zeros(1, np.uint64)  # (get_batch_dev's "needed" word, kept: one allocation less per call)
        self._need_p = _ptr(self._need)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.px_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def trim(self, keep_bytes: int = 0) -> None:
        """Give cached free device memory back to the driver (px_trim)."""
        rc = self._lib.px_trim(self._h, int(keep_bytes))
        if rc != PX_OK:
            raise PxError(rc, "px_trim")

    @property
    def stream(self) -> int:
        return self._lib.px_stream(self._h) or 0

    # ------------------------------------------------------------ setitem
    def set_batch(self, keys, vals=None, *, check: bool = True) -> np.ndarray:
        """Host inputs: lists of bytes (or (buf, off) CSR pairs).  Returns set results."""
        kb, ko = keys if isinstance(keys, tuple) else csr(keys)
        if vals is None:
            vals = [b""] * (len(ko) - 1)
        vb, vo = vals if isinstance(vals, tuple) else csr(vals)
        kb, ko, vb, vo = (np.ascontiguousarray(kb, np.uint8), np.ascontiguousarray(ko, np.uint64),
                          np.ascontiguousarray(vb, np.uint8), np.ascontiguousarray(vo, np.uint64))
        n = len(ko) - 1
        res = np.zeros(n, SET_RESULT_DTYPE)
        rc = self._lib.px_set_batch(self._h, n, _ptr(kb), _ptr(ko), _ptr(vb), _ptr(vo), 0, _ptr(res))
        if check and rc != PX_OK:
            raise PxError(rc, "px_set_batch")
        return res

    def set_docs(self, docs, reinsert: bool = False, *, check: bool = True) -> np.ndarray:
        """Ready escaped docs (PiXiuCtrl::setitem(k, 0, NULL, 0, reinsert)): list of bytes."""
        db, do = docs if isinstance(docs, tuple) else csr(docs)
        db, do = np.ascontiguousarray(db, np.uint8), np.ascontiguousarray(do, np.uint64)
        n = len(do) - 1
        res = np.zeros(n, SET_RESULT_DTYPE)
        rc = self._lib.px_set_docs(self._h, n, _ptr(db), _ptr(do), 0, int(reinsert), _ptr(res))
        if check and rc != PX_OK:
            raise PxError(rc, "px_set_docs")
        return res

    def flush(self) -> np.ndarray:
        """Store the write-behind queue; returns the last stored record's result (1 entry)."""
        res = np.zeros(1, SET_RESULT_DTYPE)
        rc = self._lib.px_flush(self._h, _ptr(res))
        if rc != PX_OK:
            raise PxError(rc, "px_flush")
        return res

    def set_batch_device(self, n: int, keys_ptr: int, koff_ptr: int, vals_ptr: int, voff_ptr: int,
                         *, check: bool = True) -> np.ndarray:
        """Inputs already resident in HBM (device pointers, e.g. torch tensor data_ptr())."""
        res = np.zeros(n, SET_RESULT_DTYPE)
        rc = self._lib.px_set_batch(self._h, n, keys_ptr, koff_ptr, vals_ptr, voff_ptr, 1, _ptr(res))
        if check and rc != PX_OK:
            raise PxError(rc, "px_set_batch")
        return res

    # ------------------------------------------------------------ getitem
    def _expand(self, fn, n, args, out_dev_ptr, out_cap, into=None):
        if into is not None:  # caller-owned (offsets u64, lengths u32, statuses u32) of >= n entries
            off, ln, st = into
            if len(off) < n or len(ln) < n or len(st) < n or off.dtype != np.uint64 or ln.dtype != np.uint32 \
                    or st.dtype != np.uint32 or not all(a.flags.c_contiguous for a in (off, ln, st)):
                raise ValueError("into: C-contiguous uint64 / uint32 / uint32 arrays of >= n entries")
        else:
            off = np.zeros(max(n, 1), np.uint64)
            ln = np.zeros(max(n, 1), np.uint32)
            st = np.zeros(max(n, 1), np.uint32)
        need = np.zeros(1, np.uint64)
        if out_dev_ptr is not None:
            rc = fn(self._h, n, *args, out_dev_ptr, out_cap, 1, _ptr(off), _ptr(ln), _ptr(st), _ptr(need))
            return rc, None, off[:n], ln[:n], st[:n], int(need[0])
        cap = 1 << 16
        while True:
            out = np.zeros(cap, np.uint8)
            rc = fn(self._h, n, *args, _ptr(out), cap, 0, _ptr(off), _ptr(ln), _ptr(st), _ptr(need))
            if rc == PX_ESPACE and int(need[0]) > cap:
                cap = int(need[0])
                continue
            return rc, out, off[:n], ln[:n], st[:n], int(need[0])

    def get_batch(self, keys, mode: int = COMPAT):
        """List of bytes (None where the key is missing), like draining PiXiuCtrl::getitem."""
        kb, ko = keys if isinstance(keys, tuple) else csr(keys)
        n = len(ko) - 1
        rc, out, off, ln, st, _ = self._expand(self._lib.px_get_batch, n, (_ptr(kb), _ptr(ko), mode), None, 0)
        res = []
        for i in range(n):
            if st[i] == PX_ENOTFOUND:
                res.append(None)
            elif st[i] != PX_OK:
                raise PxError(int(st[i]), f"getitem[{i}]")
            else:
                res.append(out[int(off[i]):int(off[i]) + int(ln[i])].tobytes())
        return res

    def get_batch_device(self, keys, out_ptr: int, out_cap: int, mode: int = COMPAT, into=None):
        """Expand into a device buffer; returns (rc, offsets, lengths, statuses, needed).
        into: optional (offsets, lengths, statuses) host arrays to fill (reused by a caller that
        repeats batches: fresh result arrays cost a page fault per 4 KB on first write)."""
        kb, ko = keys if isinstance(keys, tuple) else csr(keys)
        n = len(ko) - 1
        rc, _, off, ln, st, need = self._expand(self._lib.px_get_batch, n, (_ptr(kb), _ptr(ko), mode),
                                                out_ptr, out_cap, into)
        return rc, off, ln, st, need

    def get_batch_dev(self, n: int, keys_ptr: int, koff_ptr: int, out_ptr: int, out_cap: int, off_ptr: int,
                      len_ptr: int, status_ptr: int, mode: int = COMPAT):
        """getitem with device-resident keys (CSR: bytes + n + 1 u64 offsets) and results (u64
        offsets, u32 lengths, u32 statuses, n each): px_get_batch_dev.  Returns (rc, needed)."""
        rc = self._lib.px_get_batch_dev(self._h, n, keys_ptr, koff_ptr, mode, out_ptr, out_cap, off_ptr, len_ptr,
                                        status_ptr, self._need_p)
        return rc, int(self._need[0])

    def get_batch_host(self, keys, out: np.ndarray, mode: int = COMPAT):
        """Expand into a caller-owned host buffer (one call, no retry); returns
        (rc, offsets, lengths, statuses, needed) like get_batch_device."""
        kb, ko = keys if isinstance(keys, tuple) else csr(keys)
        n = len(ko) - 1
        off = np.zeros(max(n, 1), np.uint64)
        ln = np.zeros(max(n, 1), np.uint32)
        st = np.zeros(max(n, 1), np.uint32)
        need = np.zeros(1, np.uint64)
        rc = self._lib.px_get_batch(self._h, n, _ptr(kb), _ptr(ko), mode, _ptr(out), out.nbytes, 0,
                                    _ptr(off), _ptr(ln), _ptr(st), _ptr(need))
        return rc, off[:n], ln[:n], st[:n], int(need[0])

    def parse_batch(self, recs: np.ndarray, mode: int = COMPAT, out_ptr: int | None = None, out_cap: int = 0):
        """PiXiuStr::parse(from, to) of stored records (REC_DTYPE array)."""
        recs = np.ascontiguousarray(recs, REC_DTYPE)
        n = len(recs)
        rc, out, off, ln, st, need = self._expand(self._lib.px_parse_batch, n, (_ptr(recs), mode), out_ptr, out_cap)
        if out_ptr is not None:
            return rc, off, ln, st, need
        return [out[int(off[i]):int(off[i]) + int(ln[i])].tobytes() if st[i] == PX_OK else int(st[i])
                for i in range(n)]

    def contains(self, keys) -> np.ndarray:
        kb, ko = keys if isinstance(keys, tuple) else csr(keys)
        n = len(ko) - 1
        r = np.zeros(max(n, 1), np.uint32)
        rc = self._lib.px_contains_batch(self._h, n, _ptr(kb), _ptr(ko), _ptr(r))
        if rc != PX_OK:
            raise PxError(rc, "px_contains_batch")
        return r[:n].astype(bool)

    def delete(self, keys) -> np.ndarray:
        kb, ko = keys if isinstance(keys, tuple) else csr(keys)
        n = len(ko) - 1
        r = np.zeros(max(n, 1), np.uint32)
        rc = self._lib.px_del_batch(self._h, n, _ptr(kb), _ptr(ko), _ptr(r))
        if rc != PX_OK:
            raise PxError(rc, "px_del_batch")
        return r[:n]

    def locate(self, keys):
        """The record each key resolves to (REC_DTYPE, parse range [0, 65535)) and its status
        (PX_OK / PX_ENOTFOUND): getitem's lookup without the expansion."""
        kb, ko = keys if isinstance(keys, tuple) else csr(keys)
        n = len(ko) - 1
        recs = np.zeros(max(n, 1), REC_DTYPE)
        st = np.zeros(max(n, 1), np.uint32)
        rc = self._lib.px_locate_batch(self._h, n, _ptr(kb), _ptr(ko), _ptr(recs), _ptr(st))
        if rc != PX_OK:
            raise PxError(rc, "px_locate_batch")
        return recs[:n], st[:n]

    def reinsert(self, shard: int, chunk: int):
        """PiXiuCtrl::reinsert(PiXiuChunk *&) on a closed slot-full chunk (PiXiuCtrl.cpp:88-114)."""
        rc = self._lib.px_reinsert(self._h, shard, chunk)
        if rc != PX_OK:
            raise PxError(rc, "px_reinsert")

    def iter(self, prefix: bytes):
        """PiXiuCtrl::iter: the yielded records (REC_DTYPE, yield order), or None when every
        tree is empty (the reference's NULL generator).  Expand with parse_batch."""
        pb = np.frombuffer(prefix, np.uint8) if prefix else np.zeros(1, np.uint8)
        n = C.c_uint32(0)
        cap = 1024
        while True:
            recs = np.zeros(cap, REC_DTYPE)
            rc = self._lib.px_iter(self._h, _ptr(pb), len(prefix), _ptr(recs), cap, C.byref(n))
            if rc == PX_ESPACE:
                cap = n.value
                continue
            if rc == PX_ENOTFOUND:
                return None
            if rc != PX_OK:
                raise PxError(rc, "px_iter")
            return recs[:n.value]

    def export(self, recs: np.ndarray) -> list:
        recs = np.ascontiguousarray(recs, REC_DTYPE)
        n = len(recs)
        cap = 70000 * max(n, 1)
        out = np.zeros(cap, np.uint8)
        off = np.zeros(n + 1, np.uint64)
        rc = self._lib.px_export(self._h, n, _ptr(recs), _ptr(out), cap, _ptr(off))
        if rc != PX_OK:
            raise PxError(rc, "px_export")
        return [out[int(off[i]):int(off[i + 1])].tobytes() for i in range(n)]

    def import_chunk(self, recs: list) -> int:
        """Load compressed records as one chunk of a new read-only shard; returns the shard id."""
        buf, off = csr(recs)
        sid = np.zeros(1, np.uint32)
        rc = self._lib.px_import_chunk(self._h, len(recs), _ptr(buf), _ptr(off), _ptr(sid))
        if rc != PX_OK:
            raise PxError(rc, "px_import_chunk")
        return int(sid[0])

    # ------------------------------------------------------------ chunk blob (v1)
    def save(self) -> bytes:
        """Every stored chunk as one blob (include/pixiu_amd.h; pixiu_amd/blob.py reads it)."""
        b = np.zeros(1, np.uint64)
        rc = self._lib.px_save(self._h, None, 0, 0, _ptr(b))
        if rc != PX_OK:
            raise PxError(rc, "px_save")
        out = np.zeros(max(int(b[0]), 1), np.uint8)
        rc = self._lib.px_save(self._h, _ptr(out), out.nbytes, 0, _ptr(b))
        if rc != PX_OK:
            raise PxError(rc, "px_save")
        return out[:int(b[0])].tobytes()

    def save_device(self, dst_ptr: int, cap: int) -> int:
        """Write the blob into a device buffer; returns its size (cap 0: size only)."""
        b = np.zeros(1, np.uint64)
        rc = self._lib.px_save(self._h, dst_ptr if cap else None, cap, 1, _ptr(b))
        if rc != PX_OK:
            raise PxError(rc, "px_save")
        return int(b[0])

    def load(self, blob, on_device: bool = False, length: int = 0) -> int:
        """Add a blob's chunks (host bytes, or a device pointer + length); returns the
        first new shard id."""
        sid = np.zeros(1, np.uint32)
        if on_device:
            rc = self._lib.px_load(self._h, blob, length, 1, _ptr(sid))
        else:
            buf = np.frombuffer(blob, np.uint8)
            rc = self._lib.px_load(self._h, _ptr(buf), buf.nbytes, 0, _ptr(sid))
        if rc != PX_OK:
            raise PxError(rc, "px_load")
        return int(sid[0])

    def reset(self):
        """Drop all records, keep device memory (free_prop + init_prop)."""
        rc = self._lib.px_reset(self._h)
        if rc != PX_OK:
            raise PxError(rc, "px_reset")

    def last_store_bytes(self) -> int:
        b = np.zeros(1, np.uint64)
        self._lib.px_last_store(self._h, None, 0, 0, _ptr(b))
        return int(b[0])

    def copy_last_store(self, dst_ptr: int, cap: int, on_device: bool = True) -> int:
        b = np.zeros(1, np.uint64)
        rc = self._lib.px_last_store(self._h, dst_ptr, cap, int(on_device), _ptr(b))
        if rc != PX_OK:
            raise PxError(rc, "px_last_store")
        return int(b[0])

    def stats(self) -> dict:
        s = PxStats()
        self._lib.px_stats_get(self._h, C.byref(s))
        return {k: getattr(s, k) for k, _ in PxStats._fields_}


def records_of(res: np.ndarray, frm: int = 0, to: int = 65535) -> np.ndarray:
    """set_batch results -> REC_DTYPE array addressing those records."""
    r = np.zeros(len(res), REC_DTYPE)
    r["shard"], r["chunk"], r["idx"] = res["shard"], res["chunk"], res["idx"]
    r["from"], r["to"] = frm, to
    return r
