"""PiXiuCtrl::iter (CritBitTree.h:55-157): the oracle's restatement against the
reference built from its own sources (build container only), plus the reference's
own t_CritBitTree / t_PiXiuCtrl iteration properties (sorted keys under a prefix,
nothing for an absent prefix, NULL for an empty tree) checked on the oracle alone."""
import ctypes as C
import os
import random

import pytest

from _oracle import COMPAT, Oracle, Reference, have_reference

ALPHA = [b"A", b"B", b"C", b"D", b"E"]


def ops_for(seed, n=300):
    """t_CritBitTree-style workload: random keys over A-E + '.', random deletes."""
    rng = random.Random(seed)
    live, ops = {}, []
    for i in range(n):
        k = b"".join(rng.choice(ALPHA) for _ in range(rng.randint(0, 9))) + b"."
        v = bytes(rng.randint(33, 126) for _ in range(rng.randint(0, 40)))
        if seed % 3 == 0 and rng.random() < 0.1:
            v += bytes([251]) * rng.randint(1, 3)  # escape bytes in values
        ops.append(("set", k, v))
        live[k] = v
        if rng.random() < 0.4:
            kd = rng.choice(sorted(live))
            ops.append(("del", kd, b""))
            del live[kd]
    return ops, live


PREFIXES = [b"", b"A", b"C", b"CA", b"EEE", b"F", b"A.", b"B" * 9 + b".", bytes([251])]


def oracle_iter(ops, prefixes):
    sh = Oracle().new()
    for op, k, v in ops:
        if op == "set":
            rc, _, _ = sh.set(k, v)
            assert rc >= 0
        else:
            sh.delete(k)
    res = {}
    for p in prefixes:
        recs = sh.iter(p)
        res[p] = None if recs is None else [sh.parse(c, i, 0, 65535, COMPAT) for c, i in recs]
    return res


def ref_iter_child(ops, prefixes):
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:
        os.close(r)
        import faulthandler
        faulthandler.disable()
        try:
            lib = Reference().lib
            lib.refx_init()
            cn, ix = C.c_uint32(), C.c_uint32()
            for op, k, v in ops:
                if op == "set":
                    lib.refx_setitem(k, len(k), v, len(v), C.byref(cn), C.byref(ix))
                else:
                    lib.refx_delitem(k, len(k))
            res = {}
            buf = C.create_string_buffer(1 << 24)
            off = (C.c_uint64 * 100001)()
            for p in prefixes:
                n = lib.refx_iter(p, len(p), buf, len(buf), off, 100000)
                if n == -1:
                    res[p] = None
                else:
                    assert n >= 0
                    res[p] = [buf.raw[off[i]:off[i + 1]] for i in range(n)]
            data = repr(res).encode()
        except Exception as e:  # noqa: BLE001
            data = b"ERR" + repr(e).encode()
        with os.fdopen(w, "wb") as f:
            f.write(data)
        os._exit(0)
    os.close(w)
    with os.fdopen(r, "rb") as f:
        data = f.read()
    _, st = os.waitpid(pid, 0)
    assert not os.WIFSIGNALED(st) and not data.startswith(b"ERR"), data[:200]
    return eval(data.decode())


def test_iter_properties():
    """t_CritBitTree <遍历>: records under a prefix come out in key order; none for 'F'."""
    ops, live = ops_for(11)
    got = oracle_iter(ops, [b"C", b"F", b""])
    want = [k for k in sorted(live) if k.startswith(b"C")]
    assert [d.split(b"\xfb\x00")[0] for d in got[b"C"]] == want
    assert got[b"F"] == []
    assert [d.split(b"\xfb\x00")[0] for d in got[b""]] == sorted(live)
    empty = oracle_iter([], [b"A"])
    assert empty[b"A"] is None  # iter on an empty tree returns NULL


@pytest.mark.skipif(not have_reference(), reason="reference build not present")
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_iter_vs_reference(seed):
    ops, _ = ops_for(seed)
    assert oracle_iter(ops, PREFIXES) == ref_iter_child(ops, PREFIXES)
