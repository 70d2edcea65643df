"""Differential fuzz: the clean-room oracle against the reference built from its
own sources (build container only; skipped where /root/reference is absent).
Inputs on which the reference crashes (its GST dereferences NULL) must make the
oracle report an error instead."""
import os
import random

import pytest

from _oracle import Oracle, Reference, have_reference

pytestmark = pytest.mark.skipif(not have_reference(), reason="reference build not present")

ALPHAS = [b"ab", b"abc", b"ABCDE", bytes([97, 98, 251]), bytes([251, 0, 2, 1, 97]), bytes(range(256)),
          b"abcdefghij", b"<div></div>href=0123456789"]


def gen(rng, n, alpha, kmax, vmax):
    keys, vals, seen = [], [], set()
    while len(keys) < n:
        k = bytes(rng.choice(alpha) for _ in range(rng.randint(1, kmax)))
        if k in seen:
            continue
        seen.add(k)
        keys.append(k)
        vals.append(bytes(rng.choice(alpha) for _ in range(rng.randint(0, vmax))))
    return keys, vals


def ref_in_child(keys, vals):
    """Run the reference in a forked child: it may segfault (UB / NULL deref)."""
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:
        os.close(r)
        import faulthandler
        faulthandler.disable()  # an expected crash of the reference: no traceback spam
        try:
            out = Reference().run(keys, vals)
            data = repr((out["comp"], out["chunk"], out["idx"], out["get"])).encode()
        except Exception:
            data = b"ERR"
        with os.fdopen(w, "wb") as f:
            f.write(data)
        os._exit(0)
    os.close(w)
    with os.fdopen(r, "rb") as f:
        data = f.read()
    _, st = os.waitpid(pid, 0)
    if os.WIFSIGNALED(st) or data in (b"", b"ERR"):
        return None
    return eval(data.decode())  # our own child's repr of bytes/ints


@pytest.mark.parametrize("seed", list(range(1, 7)))
def test_fuzz(seed):
    rng = random.Random(seed)
    orc = Oracle()
    eq = crash = 0
    for _ in range(60):
        keys, vals = gen(rng, rng.randint(1, 30), rng.choice(ALPHAS), 6, rng.choice([5, 30, 200, 1000]))
        try:
            o = orc.run(keys, vals)
            mine = (o["comp"], o["chunk"], o["idx"], o["get"])
        except RuntimeError:
            mine = None
        ref = ref_in_child(keys, vals)
        if ref is None:
            assert mine is None, "reference crashed but the oracle did not flag the input"
            crash += 1
            continue
        assert mine == ref
        eq += 1
    assert eq > 40
