#!/usr/bin/env python3
"""Generate tests/golden/ from the REFERENCE ITSELF (oracle/_ref/libpxref.so, built
from /root/reference/src by `make -C oracle ref`).  Run in the build container
only; the outputs are data (inputs + expected outputs), never reference source.

    python tools/make_golden.py            # writes tests/golden/*

Fixtures:
  kats.json          escape / stream-encoder / hand-built-chunk decoder KATs
                     (PiXiuStr.cpp:301-413 shapes), README transcript (README.md:71-95),
                     decoder-bug and len-251 repros, max-size records
                     (PiXiuCtrl.cpp:121-174), a randomized CRUD script (PiXiuCtrl.cpp:176-226 shape)
  corpus_c{1..5}.npz per-config mini corpora: compressed bytes, chunk/slot, compat getitem
  rotation.json      >= 12 MB single-shard corpora crossing a chunk rotation (pool count
                     and slot count): per-chunk record counts + sha256 of every chunk's bytes
  reinsert.json      slot-full chunks compacted by reinsert (PiXiuCtrl.cpp:12-29, 63-69, 88-114):
                     digests of per-record returns and of the end state (tests/_reinsert.py)
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from pixiu_amd import synth  # noqa: E402
from _oracle import Reference, _csr, _p  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
REF = Reference()
L = REF.lib


def hx(b: bytes) -> str:
    return b.hex()


def ref_stream(msgs):
    n = len(msgs)
    cmd = (C.c_int * max(n, 1))(*[m[0] for m in msgs])
    pos = (C.c_int * max(n, 1))(*[m[1] for m in msgs])
    val = (C.c_uint8 * max(n, 1))(*[m[2] for m in msgs])
    out = C.create_string_buffer(4 * n + 64)
    r = L.refx_stream(n, cmd, pos, val, out, len(out))
    assert r >= 0
    return out.raw[:r]


def ref_escape(src: bytes, key: bool) -> bytes:
    out = C.create_string_buffer(2 * len(src) + 4)
    n = L.refx_escape(src, len(src), int(key), out)
    return out.raw[:n]


def ref_decode_chunk(recs, idx, frm, to):
    buf, off = _csr(recs)
    out = C.create_string_buffer(1 << 20)
    n = L.refx_decode_chunk(len(recs), _p(buf), _p(off), idx, frm, to, out, len(out))
    assert n >= 0, n
    return out.raw[:n]


class Live:
    """The reference's single live PiXiuCtrl."""

    def __init__(self):
        L.refx_init()

    def set(self, k, v):
        cn, ix = C.c_uint32(), C.c_uint32()
        rc = L.refx_setitem(k, len(k), v, len(v), C.byref(cn), C.byref(ix))
        buf = C.create_string_buffer(70000)
        n = L.refx_last_comp(buf, 70000)
        return rc, cn.value, ix.value, buf.raw[:n]

    def get(self, k):
        buf = C.create_string_buffer(1 << 20)
        n = L.refx_getitem(k, len(k), buf, 1 << 20)
        return None if n == -1 else buf.raw[:n]

    def contains(self, k):
        return L.refx_contains(k, len(k))

    def delete(self, k):
        return L.refx_delitem(k, len(k))


def kats():
    P = -3
    out = {}
    # escape (PiXiuStr.cpp:301-311 shape)
    src = bytes([1, 251, 2, 251, 4])
    out["escape"] = [{"src": hx(src), "key": hx(ref_escape(src, True)), "plain": hx(ref_escape(src, False))},
                     {"src": hx(b""), "key": hx(ref_escape(b"", True)), "plain": ""},
                     {"src": hx(bytes([251] * 7)), "key": hx(ref_escape(bytes([251] * 7), True)),
                      "plain": hx(ref_escape(bytes([251] * 7), False))}]
    # stream encoder (PiXiuStr.cpp:326-352 shapes + look-ahead cases)
    streams = {
        "small_record": [(P, 0, 1)] * 4 + [(2, i, 3) for i in range(6)] + [(P, 0, 1)] + [(3, i, 4) for i in range(7)],
        "big_record": [(P, 0, 1)] + [(2, i, 3) for i in range(255)] + [(P, 0, 1)] + [(3, i, 4) for i in range(256)],
        "escapes_and_records": [(P, 0, 1), (P, 0, 251), (P, 0, 251), (P, 0, 1), (1, 0, 251), (1, 1, 251), (P, 0, 3)]
        + [(2, i, 2) for i in range(11)] + [(P, 0, 3)] + [(3, i, 6) for i in range(1, 257)],
        "mixed_pair_demotes": [(P, 0, 9)] + [(4, i, 7) for i in range(8)] + [(4, 8, 251), (P, 0, 0)]
        + [(5, i, 8) for i in range(9)],
        "len_251_alias": [(P, 0, 1)] + [(6, 100 + i, 97) for i in range(251)] + [(P, 0, 1)],
        "run_6_literal": [(7, i, 65) for i in range(6)] + [(P, 0, 66)],
    }
    out["stream"] = {k: {"msgs": v, "out": hx(ref_stream(v))} for k, v in streams.items()}
    # hand-built chunk decoder KAT (PiXiuStr.cpp:356-413 shape): parse(1, 272)
    pxs = ref_stream(streams["escapes_and_records"])
    i2v2 = ref_stream([(P, 0, 2)] * 11 + [(P, 0, 8)])
    i3v6 = ref_stream([(P, 0, 8)] + [(P, 0, 6)] * 256 + [(P, 0, 8)])
    chunk = [b"\x00", pxs, i2v2, i3v6]  # slot 0 unused filler, self at slot 1
    queries = [(1, 1, 272), (1, 0, 65535), (1, 5, 20), (1, 2, 3), (1, 14, 14), (3, 10, 200)]
    out["chunk_decode"] = {"chunk": [hx(c) for c in chunk],
                           "queries": [{"idx": i, "from": a, "to": b, "out": hx(ref_decode_chunk(chunk, i, a, b))}
                                       for i, a, b in queries]}
    # README transcript (README.md:71-95): saved = len(cmd) - compressed len
    lv = Live()
    tr = []
    for cmd in ["SET 123::321", "SET BOBO::https://www.zhihu.com/question/55439090",
                "SET BOBO1::https://www.zhihu.com/question/22454692"]:
        pos = cmd.index("::")
        k, v = cmd[4:pos].encode(), cmd[pos:].encode()
        rc, cn, ix, comp = lv.set(k, v)
        tr.append({"cmd": cmd, "key": hx(k), "val": hx(v), "comp": hx(comp), "saved": len(cmd) - len(comp)})
    out["readme"] = {"steps": tr, "gets": {k: hx(lv.get(k.encode())) for k in ["123", "BOBO", "BOBO1"]}}
    assert tr[-1]["saved"] == 27
    # decoder bug repro
    lv = Live()
    recs = [lv.set(b"k0", b"abaabaabaabba"), lv.set(b"k1", b"abaababba")]
    out["decoder_bug"] = {"keys": [hx(b"k0"), hx(b"k1")], "vals": [hx(b"abaabaabaabba"), hx(b"abaababba")],
                          "comp": [hx(r[3]) for r in recs], "get_k1": hx(lv.get(b"k1"))}
    # len-251 alias
    rng = random.Random(251)
    a = bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz") for _ in range(400))
    lv = Live()
    keys, vals = [b"K1", b"K2"], [a, b"Q" + a[:251] + b"#"]
    recs = [lv.set(k, v) for k, v in zip(keys, vals)]
    out["len251"] = {"keys": [hx(k) for k in keys], "vals": [hx(v) for v in vals],
                     "comp": [hx(r[3]) for r in recs], "gets": [hx(lv.get(k)) for k in keys]}
    # max-size records (PiXiuCtrl.cpp:121-174 shapes)
    lv = Live()
    big = bytes([233]) + bytes([1]) * (65533 - 1)
    rc, cn, ix, comp = lv.set(big, b"")
    g = lv.get(big)
    out["max_elem"] = {"key": "233 then 65532 x 1", "comp_sha256": hashlib.sha256(comp).hexdigest(),
                       "comp_len": len(comp), "get_sha256": hashlib.sha256(g).hexdigest(), "get_len": len(g)}
    lv = Live()
    mk, mv = bytes([6]) * 100, bytes([2]) * (65535 - 102 - 2)
    rc, cn, ix, comp = lv.set(mk, mv)
    g = lv.get(mk)
    out["max_kv"] = {"klen": 100, "vlen": len(mv), "comp_sha256": hashlib.sha256(comp).hexdigest(),
                     "comp_len": len(comp), "get_sha256": hashlib.sha256(g).hexdigest(), "get_len": len(g)}
    # randomized CRUD script over a 5-letter alphabet (PiXiuCtrl.cpp:176-226 shape), one live instance
    rng = random.Random(19950207)
    lv = Live()
    ops = []
    live = {}
    for i in range(1500):
        k = "".join(rng.choice("ABCDE") for _ in range(rng.randint(1, 6))).encode()
        v = "".join(rng.choice("ABCDE") for _ in range(rng.randint(1, 30))).encode()
        rc, cn, ix, comp = lv.set(k, v)
        live[k] = v
        ops.append(["set", hx(k), hx(v), rc, hx(comp)])
        q = rng.choice(list(live)) if rng.random() < 0.7 else b"ZZ" + k
        g = lv.get(q)
        ops.append(["get", hx(q), None if g is None else hx(g)])
        ops.append(["contains", hx(q), lv.contains(q)])
        if rng.random() < 0.3:
            d = rng.choice(list(live)) if rng.random() < 0.8 else b"QQ"
            r = lv.delete(d)
            live.pop(d, None)
            ops.append(["del", hx(d), r])
    out["crud"] = ops
    return out


def corpora():
    spec = {1: (1000, None), 2: (64, None), 3: (8, None), 4: (2000, None), 5: (6, None)}
    for cfg, (n, _) in spec.items():
        cp = synth.make(cfg, n)
        keys = [cp.key(i) for i in range(n)]
        vals = [cp.val(i) for i in range(n)]
        r = REF.run(keys, vals, do_get=True)
        comp, coff = _csr(r["comp"])
        dec, doff = _csr(r["get"])
        h = hashlib.sha256(cp.keys.tobytes() + cp.vals.tobytes()).hexdigest()
        np.savez_compressed(os.path.join(OUT, f"corpus_c{cfg}.npz"), n=np.int64(n), comp=comp, comp_off=coff,
                            chunk=np.array(r["chunk"], np.uint32), idx=np.array(r["idx"], np.uint32),
                            get=dec, get_off=doff, input_sha256=np.frombuffer(h.encode(), np.uint8))
        print(f"corpus_c{cfg}: {n} records, comp {int(coff[-1])} B / raw {cp.raw_bytes} B")


def rotation():
    out = {}
    for name, cfg, n in [("pools_c2", 2, 14000), ("pools_c4", 4, 50000), ("slots_tiny", 0, 70000)]:
        if cfg:
            cp = synth.make(cfg, n)
        else:  # 65,535-slot rotation: tiny key-only records
            cp = synth.tiny_keys(n)
        keys = [cp.key(i) for i in range(n)]
        vals = [cp.val(i) for i in range(n)]
        r = REF.run(keys, vals, do_get=False)
        chunks = {}
        for i, c in enumerate(r["chunk"]):
            chunks.setdefault(c, []).append(i)
        per = []
        for c in sorted(chunks):
            rows = chunks[c]
            assert [r["idx"][i] for i in rows] == list(range(len(rows)))
            hsh = hashlib.sha256(b"".join(r["comp"][i] for i in rows)).hexdigest()
            per.append({"chunk": c, "first": rows[0], "records": len(rows), "sha256": hsh,
                        "comp_bytes": sum(len(r["comp"][i]) for i in rows)})
        out[name] = {"config": cfg, "n": n, "raw_bytes": cp.raw_bytes, "chunks": per,
                     "input_sha256": hashlib.sha256(cp.keys.tobytes() + cp.vals.tobytes()).hexdigest()}
        print(name, [(p["first"], p["records"]) for p in per])
    return out


def chunk_digest(r):
    """per-chunk (first record, records, sha256 of the chunk's compressed bytes in slot
    order, compressed bytes) of one instance's run"""
    chunks = {}
    for i, c in enumerate(r["chunk"]):
        chunks.setdefault(c, []).append(i)
    per = []
    for c in sorted(chunks):
        rows = chunks[c]
        assert [r["idx"][i] for i in rows] == list(range(len(rows)))
        per.append({"chunk": c, "first": rows[0], "records": len(rows),
                    "sha256": hashlib.sha256(b"".join(r["comp"][i] for i in rows)).hexdigest(),
                    "comp_bytes": sum(len(r["comp"][i]) for i in rows)})
    return per


def c3_single(runner=None, n=10000):
    """config 3 (the README shape, 10k x 60 KB) as ONE PiXiuCtrl over every page, the
    reference's own configuration (PiXiuCtrl.cpp:12-25): one row per chunk."""
    import time
    cp = synth.make(3, n)
    keys = [cp.key(i) for i in range(n)]
    vals = [cp.val(i) for i in range(n)]
    t = time.time()
    r = (runner or REF).run(keys, vals, do_get=False)
    dt = time.time() - t
    per = chunk_digest(r)
    out = {"config": 3, "n": n, "raw_bytes": cp.raw_bytes, "chunks": per,
           "comp_bytes": sum(p["comp_bytes"] for p in per),
           "input_sha256": hashlib.sha256(cp.keys.tobytes() + cp.vals.tobytes()).hexdigest(),
           "generator": type(runner or REF).__name__, "seconds": round(dt, 1)}
    print(f"c3_single: {len(per)} chunks, ratio {out['comp_bytes'] / cp.raw_bytes:.4f}, {dt:.0f} s")
    return out


def reinsert():
    """tests/_reinsert.py scenarios through the reference, one record at a time: digests
    of every record's return and of the end state (presence, compat getitem, slot,
    compressed bytes of every touched key), and where a few keys ended up."""
    import _reinsert as R
    out = {}
    for name, ops in R.scenarios().items():
        REF.init()
        rets = R.run_scalar(REF, ops)
        keys = R.touched(ops)
        state = R.reference_state(REF, keys)
        d = R.digest(rets, state)
        d["ops_sha256"] = R.ops_sha256(ops)
        d["sample"] = [[k.decode(), int(p), hx(g) if p else None, i, hx(c) if p else None]
                       for k, p, g, i, c in state[:: max(1, len(state) // 40)]]
        out[name] = d
        print(name, {k: v for k, v in d.items() if k != "sample"})
    REF.lib.refx_free()
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    what = set(sys.argv[1:]) or {"kats", "corpora", "rotation", "reinsert"}
    if "kats" in what:
        json.dump(kats(), open(os.path.join(OUT, "kats.json"), "w"))
    if "corpora" in what:
        corpora()
    if "rotation" in what:
        json.dump(rotation(), open(os.path.join(OUT, "rotation.json"), "w"), indent=1)
    if "reinsert" in what:
        json.dump(reinsert(), open(os.path.join(OUT, "reinsert.json"), "w"), indent=1)
    if "c3_single" in what:  # (not in the default set: ~13 minutes of reference time)
        json.dump(c3_single(), open(os.path.join(OUT, "c3_single.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
