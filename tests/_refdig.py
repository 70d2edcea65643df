"""Per-record digests of the REFERENCE's output at the bench's full sizes — test
infrastructure only (shared by tools/make_refdigests.py, the -m gpu tests and
bench.py's parity counts).

tests/golden/refdig_c{config}_r{rps}[_n{n}].npz holds, for every record of the canonical
corpus part (synth.make(config); _n: its first n records only) stored in records_per_shard = rps shards (one
reference PiXiuCtrl per shard, rps = 0: one over every record), in record order:

  get_len, get_d64    length and digest64 of the reference's compat getitem drain
                      (PiXiuCtrl::getitem + PXSGen, PiXiuCtrl.cpp:59-61, PiXiuStr.h:129-198)
  comp_len, comp_d64  length and digest64 of the record's compressed bytes
  chunk, idx          the chunk serial and chunk-local slot it landed in

digest64(b) = the 8-byte BLAKE2b digest of b, little-endian (round 5; the round-4 fixtures held
4-byte digests, get_d32 / comp_d32, which compare() still reads: a 2^-32 chance per record that
a wrong record matches, ~2.6e-4 over the 1.13 M records, against 2^-64 now).
"""
from __future__ import annotations

import hashlib
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def digest(b, size: int = 8) -> int:
    return int.from_bytes(hashlib.blake2b(b, digest_size=size).digest(), "little")


def digest32(b) -> int:
    return digest(b, 4)


def digest64(b) -> int:
    return digest(b, 8)


def width(ref) -> int:
    """digest bytes a fixture holds: 8 (get_d64 / comp_d64) or 4 (round 4's get_d32 / comp_d32)"""
    return 8 if "get_d64" in ref else 4


def _dig(ref, kind):
    return ref[f"{kind}_d64"] if "get_d64" in ref else ref[f"{kind}_d32"]


def digests(buf: np.ndarray, off, ln, size: int = 8) -> np.ndarray:
    """digest of buf[off[i] : off[i] + ln[i]] for every i (host buffer), `size` bytes."""
    mv = memoryview(np.ascontiguousarray(buf))
    off = np.asarray(off, np.int64).tolist()
    ln = np.asarray(ln, np.int64).tolist()
    h = hashlib.blake2b
    dt = np.uint64 if size == 8 else np.uint32
    return np.fromiter((int.from_bytes(h(mv[o:o + n], digest_size=size).digest(), "little")
                        for o, n in zip(off, ln)), dt, count=len(off))


def path(config: int, rps: int, n: int | None = None) -> str:
    """n: a fixture over only the first n records of the full corpus"""
    return os.path.join(GOLDEN, f"refdig_c{config}_r{rps}" + (f"_n{n}" if n else "") + ".npz")


def load(config: int, rps: int, n: int | None = None):
    """The reference's digests for (config, rps[, first n records]), or None without a fixture."""
    p = path(config, rps, n)
    if not os.path.exists(p):
        return None
    with np.load(p, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def compare(ref, get_len, get_dig):
    """Records whose compat getitem differs from the reference's (length or digest; get_dig
    made with the fixture's width())."""
    get_len = np.asarray(get_len, np.int64)
    want = _dig(ref, "get")
    get_dig = np.asarray(get_dig, want.dtype)
    if len(get_len) != len(ref["get_len"]):
        raise ValueError(f"{len(get_len)} records, the reference digests hold {len(ref['get_len'])}")
    bad = (get_len != ref["get_len"].astype(np.int64)) | (get_dig != want)
    return int(bad.sum()), np.nonzero(bad)[0]


def compat_all(st, keys, device):
    """Every key's compat getitem into one device buffer (pixiu_amd.Store.get_batch_device,
    grown once to the call's reported need): (buffer, offsets, lengths)."""
    import torch
    import pixiu_amd as px
    kb, ko = keys if isinstance(keys, tuple) else px.csr(keys)
    n = len(ko) - 1
    cap = int(ko[-1]) * 2 + 400 * n + (1 << 20)
    for _ in range(2):
        out = torch.empty(cap, dtype=torch.uint8, device=device)
        rc, off, ln, sts, need = st.get_batch_device((kb, ko), out.data_ptr(), cap, px.COMPAT)
        if rc == px.PX_ESPACE and need > cap:
            cap = int(need)
            continue
        if rc != px.PX_OK or (n and int(sts.max()) != 0):
            raise RuntimeError(f"compat getitem rc={rc}")
        return out, off, ln
    raise RuntimeError("compat getitem: no room")


def check_store(ref, st, res, out, off, ln):
    """A store's full-size result against the reference's digests (outside any timing).

    st, res     the pixiu_amd.Store and its set_batch results for the corpus, in record order
    out         the compat getitem output of every key in record order (a torch uint8 device
                tensor or a host numpy buffer), record i at out[off[i] : off[i] + ln[i]]
    Returns {records, compat_ne_reference, comp_ne_reference, placement_ne_reference,
    first_bad}."""
    import pixiu_amd as px
    off = np.asarray(off, np.int64)
    ln = np.asarray(ln, np.int64)
    n = len(ln)
    end = int((off + ln).max()) if n else 0
    host = out[:end].cpu().numpy() if hasattr(out, "cpu") else np.asarray(out)[:end]
    w = width(ref)
    bad_get, idx = compare(ref, ln, digests(host, off, ln, w))
    comp = st.export(px.records_of(res))
    cl = np.fromiter((len(c) for c in comp), np.int64, count=n)
    cd = np.fromiter((digest(c, w) for c in comp), np.uint64 if w == 8 else np.uint32, count=n)
    bad_comp = int(((cl != ref["comp_len"].astype(np.int64)) | (cd != _dig(ref, "comp"))).sum())
    bad_place = int(((np.asarray(res["chunk"], np.int64) != ref["chunk"].astype(np.int64))
                     | (np.asarray(res["idx"], np.int64) != ref["idx"].astype(np.int64))).sum())
    return {"records": n, "compat_ne_reference": bad_get, "comp_ne_reference": bad_comp,
            "placement_ne_reference": bad_place, "first_bad": [int(i) for i in idx[:5]], "digest_bits": 8 * w}
