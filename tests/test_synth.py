"""Synthetic corpora are deterministic and have the §8(d) shapes."""
import hashlib

import numpy as np

from pixiu_amd import synth


def digest(cp):
    return hashlib.sha256(cp.keys.tobytes() + cp.vals.tobytes()).hexdigest()


def test_deterministic():
    for cfg, n in [(1, 50), (2, 20), (3, 3), (4, 100), (5, 2)]:
        assert digest(synth.make(cfg, n)) == digest(synth.make(cfg, n))


def test_shapes():
    c3 = synth.make(3, 4)
    assert all(c3.voff[i + 1] - c3.voff[i] == 60000 for i in range(4))
    assert c3.key(0).startswith(b"http://www.qq.com/a/2017")
    v = c3.vals
    assert v.min() >= 33 and v.max() <= 126  # visible ASCII only (README.md:51)
    c4 = synth.make(4, 1000)
    frac = float((c4.vals == 251).mean())
    assert 0.08 < frac < 0.12
    c5 = synth.make(5, 3)
    assert all(c5.koff[i + 1] - c5.koff[i] + c5.voff[i + 1] - c5.voff[i] == 65531 for i in range(3))
    assert not (c5.vals == 251).any()


def test_parts_are_independent():
    a, b = synth.make(3, 2), synth.make(3, 2, part=1)
    assert a.key(0) != b.key(0)
    assert not np.array_equal(a.vals, b.vals)
