"""ctypes access to the CPU checker (oracle/) — TEST INFRASTRUCTURE ONLY.

``Oracle`` wraps oracle/_build/libpxo.so, the clean-room restatement (oracle/pxo.cpp).
``Reference`` wraps oracle/_ref/libpxref.so, the reference compiled from its own
sources; it exists only in the build container (never on the GPU box).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PXO_LIB: another build of the same restatement (the sanitizer build, oracle/Makefile asan)
ORACLE_SO = os.environ.get("PXO_LIB") or os.path.join(ROOT, "oracle", "_build", "libpxo.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libpxref.so")

COMPAT, EXACT = 0, 1
PXO_NOTFOUND = -5


def build_oracle() -> str:
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return ORACLE_SO


def _csr(items):
    lens = np.fromiter((len(x) for x in items), dtype=np.uint64, count=len(items))
    off = np.zeros(len(items) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    buf = np.frombuffer(b"".join(items), np.uint8).copy() if items else np.zeros(0, np.uint8)
    return (buf if buf.size else np.zeros(1, np.uint8)), off


def _p(a):
    return C.c_void_p(a.ctypes.data)


class _Runner:
    lib: C.CDLL
    run_fn: str
    has_mode: bool

    def run(self, keys, vals, do_get=True, mode=COMPAT):
        """Insert all records into one fresh instance; returns dict of per-record results."""
        n = len(keys)
        kb, ko = _csr(keys)
        vb, vo = _csr(vals)
        kl = np.diff(ko).astype(np.uint32)
        vl = np.diff(vo).astype(np.uint32)
        ko64 = ko[:-1].copy()
        vo64 = vo[:-1].copy()
        raw = int(ko[-1] + vo[-1])
        cap = 2 * raw + 16 * n + 1024
        comp = np.zeros(cap, np.uint8)
        coff = np.zeros(n + 1, np.uint64)
        ch = np.zeros(max(n, 1), np.uint32)
        ix = np.zeros(max(n, 1), np.uint32)
        dcap = 4 * cap + (1 << 16)
        dec = np.zeros(dcap, np.uint8)
        doff = np.zeros(n + 1, np.uint64)
        args = [C.c_int(n), _p(kb), _p(ko64), _p(kl), _p(vb), _p(vo64), _p(vl), _p(comp), C.c_uint64(cap),
                _p(coff), _p(ch), _p(ix), C.c_int(1 if do_get else 0)]
        if self.has_mode:
            args.append(C.c_int(mode))
        args += [_p(dec), C.c_uint64(dcap), _p(doff)]
        rc = getattr(self.lib, self.run_fn)(*args)
        if rc != 0:
            raise RuntimeError(f"{self.run_fn} failed: {rc}")
        out = {
            "comp": [comp[coff[i]:coff[i + 1]].tobytes() for i in range(n)],
            "chunk": ch[:n].tolist(),
            "idx": ix[:n].tolist(),
        }
        if do_get:
            out["get"] = [dec[doff[i]:doff[i + 1]].tobytes() for i in range(n)]
        return out


class Oracle(_Runner):
    def __init__(self):
        self.lib = C.CDLL(build_oracle())
        self.lib.pxo_new.restype = C.c_void_p
        self.lib.pxo_free.argtypes = [C.c_void_p]
        self.lib.pxo_ub_reads.restype = C.c_long
        self.run_fn = "pxo_run"
        self.has_mode = True

    def encode_docs(self, docs):
        """Encoder only, over already-assembled docs (one shard)."""
        n = len(docs)
        db, do = _csr(docs)
        cap = int(do[-1]) + 64
        comp = np.zeros(cap, np.uint8)
        coff = np.zeros(n + 1, np.uint64)
        ch = np.zeros(max(n, 1), np.uint32)
        ix = np.zeros(max(n, 1), np.uint32)
        rc = self.lib.pxo_encode_docs(C.c_int(n), _p(db), _p(do), _p(comp), C.c_uint64(cap), _p(coff), _p(ch), _p(ix))
        if rc != 0:
            raise RuntimeError(f"pxo_encode_docs failed: {rc}")
        return [comp[coff[i]:coff[i + 1]].tobytes() for i in range(n)], ch[:n].tolist(), ix[:n].tolist()

    def decode_chunk(self, recs, idx, frm=0, to=65535, mode=COMPAT) -> bytes:
        """PiXiuStr::parse(frm, to) of record idx of a chunk given as compressed bytes."""
        buf, off = _csr(list(recs))
        out = C.create_string_buffer(1 << 20)
        r = self.lib.pxo_decode_chunk(C.c_int(len(recs)), _p(buf), _p(off), C.c_int(idx), C.c_int(frm),
                                      C.c_int(to), C.c_int(mode), out, C.c_int(len(out)))
        if r < 0:
            raise RuntimeError(f"pxo_decode_chunk: {r}")
        return out.raw[:r]

    def escape(self, src: bytes, is_key: bool) -> bytes:
        out = C.create_string_buffer(2 * len(src) + 4)
        n = self.lib.pxo_escape(src, len(src), int(is_key), out, len(out))
        return out.raw[:n]

    def stream(self, msgs) -> bytes:
        """msgs: list of (cmd, pos, val); cmd >= 0 compress, -3 pass."""
        n = len(msgs)
        cmd = (C.c_int * max(n, 1))(*[m[0] for m in msgs])
        pos = (C.c_int * max(n, 1))(*[m[1] for m in msgs])
        val = (C.c_uint8 * max(n, 1))(*[m[2] for m in msgs])
        out = C.create_string_buffer(4 * n + 64)
        r = self.lib.pxo_stream(n, cmd, pos, val, out, len(out))
        if r < 0:
            raise RuntimeError(f"pxo_stream: {r}")
        return out.raw[:r]

    # incremental handle API
    def new(self):
        return _Shard(self.lib)


class _Shard:
    def __init__(self, lib):
        self.lib = lib
        self.h = C.c_void_p(lib.pxo_new())

    def __del__(self):
        try:
            self.lib.pxo_free(self.h)
        except Exception:
            pass

    def set(self, k: bytes, v: bytes):
        cn, ix = C.c_uint32(), C.c_uint32()
        rc = self.lib.pxo_set(self.h, k, len(k), v, len(v), C.byref(cn), C.byref(ix))
        return rc, cn.value, ix.value

    def get(self, k: bytes, mode=COMPAT):
        out = C.create_string_buffer(1 << 20)
        n = self.lib.pxo_get(self.h, k, len(k), mode, out, len(out))
        if n == PXO_NOTFOUND:
            return None
        if n < 0:
            raise RuntimeError(f"pxo_get: {n}")
        return out.raw[:n]

    def parse(self, chunk, idx, frm, to, mode=COMPAT):
        out = C.create_string_buffer(1 << 20)
        n = self.lib.pxo_parse(self.h, chunk, idx, frm, to, mode, out, len(out))
        if n < 0:
            raise RuntimeError(f"pxo_parse: {n}")
        return out.raw[:n]

    def contains(self, k: bytes) -> int:
        return self.lib.pxo_contains(self.h, k, len(k))

    def iter(self, prefix: bytes):
        """PiXiuCtrl::iter: [(chunk, idx)] in yield order, None for an empty tree."""
        cap = 1 << 20
        ch = (C.c_uint32 * cap)()
        ix = (C.c_uint32 * cap)()
        n = self.lib.pxo_iter(self.h, prefix, len(prefix), ch, ix, cap)
        if n == PXO_NOTFOUND:
            return None
        if n < 0:
            raise RuntimeError(f"pxo_iter: {n}")
        return [(ch[i], ix[i]) for i in range(n)]

    def delete(self, k: bytes) -> int:
        return self.lib.pxo_delete(self.h, k, len(k))

    def reinsert(self, chunk: int) -> int:
        """PiXiuCtrl::reinsert(PiXiuChunk *&) on closed chunk `chunk` (PiXiuCtrl.cpp:88-114)"""
        return self.lib.pxo_reinsert(self.h, chunk)

    def locate(self, k: bytes):
        """(chunk, idx) of the key's record, or None."""
        cn, ix = C.c_uint32(), C.c_uint32()
        rc = self.lib.pxo_locate(self.h, k, len(k), C.byref(cn), C.byref(ix))
        if rc == PXO_NOTFOUND:
            return None
        if rc < 0:
            raise RuntimeError(f"pxo_locate: {rc}")
        return cn.value, ix.value

    def comp(self, chunk, idx):
        out = C.create_string_buffer(1 << 17)
        n = self.lib.pxo_comp(self.h, chunk, idx, out, len(out))
        return out.raw[:n]

    def ub_reads(self):
        return self.lib.pxo_ub_reads(self.h)


class Reference(_Runner):
    """The reference itself (build container only)."""

    def __init__(self):
        if not os.path.exists(REF_SO):
            raise FileNotFoundError(REF_SO)
        self.lib = C.CDLL(REF_SO)
        self.run_fn = "refx_run"
        self.has_mode = False

    # incremental API over the library's single global controller (PiXiuCtrl.cpp:12-69)
    def init(self):
        self.lib.refx_init()
        return self

    def set(self, k: bytes, v: bytes) -> int:
        cn, ix = C.c_uint32(), C.c_uint32()
        return self.lib.refx_setitem(k, len(k), v, len(v), C.byref(cn), C.byref(ix))

    def delete(self, k: bytes) -> int:
        return self.lib.refx_delitem(k, len(k))

    def reinsert(self, chunk: int) -> int:
        return self.lib.refx_reinsert(chunk)

    def contains(self, k: bytes) -> int:
        return self.lib.refx_contains(k, len(k))

    def get(self, k: bytes):
        out = C.create_string_buffer(1 << 17)
        n = self.lib.refx_getitem(k, len(k), out, len(out))
        if n == -1:
            return None
        if n < 0:
            raise RuntimeError(f"refx_getitem: {n}")
        return out.raw[:n]

    def locate_comp(self, k: bytes):
        """(idx, compressed bytes) of the key's record, or None."""
        out = C.create_string_buffer(1 << 17)
        ix = C.c_uint32()
        n = self.lib.refx_locate(k, len(k), out, len(out), C.byref(ix))
        if n == -5:
            return None
        if n < 0:
            raise RuntimeError(f"refx_locate: {n}")
        return ix.value, out.raw[:n]


def have_reference() -> bool:
    """The reference build, made on demand from /root/reference/src (build container
    only: the GPU box has no reference, and oracle/_ref never travels there)."""
    if not os.path.isdir("/root/reference/src"):
        return False
    if not os.path.exists(REF_SO):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=False)
    return os.path.exists(REF_SO)


def assemble(k: bytes, v: bytes) -> bytes:
    """Escaped doc (PiXiuCtrl.cpp:31-44) in pure Python, for small cases."""
    def esc(x):
        return x.replace(b"\xfb", b"\xfb\xfb")
    d = esc(k) + b"\xfb\x00"
    if v:
        d += esc(v) + b"\xfb\x02"
    return d
