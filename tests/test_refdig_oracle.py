"""The reference's full-size digests (tests/golden/refdig_*.npz) against the CPU oracle on
each fixture's leading records (CPU only).  A record's compressed bytes, placement and
compat getitem depend only on the records before it in its shard (references point back
into the same chunk; keys are unique), so the oracle over a shard's first k records must
reproduce the fixture's first k rows exactly."""
import numpy as np
import pytest

import _refdig

LEAD = {2: 1500, 3: 24, 4: 3000, 5: 24}
CASES = [(2, 2000), (3, 139), (3, 0), (4, 8000), (5, 126)]


@pytest.mark.parametrize("cfg,rps", CASES, ids=[f"c{c}_rps{r}" for c, r in CASES])
def test_oracle_reproduces_reference_digest_prefix(cfg, rps, oracle):
    ref = _refdig.load(cfg, rps)
    if ref is None:
        pytest.skip(f"no fixture {_refdig.path(cfg, rps)}")
    from pixiu_amd import synth
    k = LEAD[cfg]
    cp = synth.make(cfg)  # (the full corpus: a generator's draws depend on its record count)
    r = oracle.run([cp.key(i) for i in range(k)], [cp.val(i) for i in range(k)])
    w = _refdig.width(ref)
    d = lambda b: _refdig.digest(b, w)  # noqa: E731
    dk = "d64" if w == 8 else "d32"
    assert [len(g) for g in r["get"]] == ref["get_len"][:k].tolist()
    assert [d(g) for g in r["get"]] == ref[f"get_{dk}"][:k].tolist()
    assert [len(c) for c in r["comp"]] == ref["comp_len"][:k].tolist()
    assert [d(c) for c in r["comp"]] == ref[f"comp_{dk}"][:k].tolist()
    assert r["chunk"] == ref["chunk"][:k].tolist() and r["idx"] == ref["idx"][:k].tolist()


def test_fixture_shapes():
    for cfg, rps in CASES:
        ref = _refdig.load(cfg, rps)
        if ref is None:
            continue
        n = int(ref["n"])
        dk = "d64" if _refdig.width(ref) == 8 else "d32"
        for f in ("get_len", f"get_{dk}", "comp_len", f"comp_{dk}", "chunk", "idx"):
            assert ref[f].shape == (n,), (cfg, rps, f)
        assert ref[f"get_{dk}"].dtype == (np.uint64 if dk == "d64" else np.uint32)
        assert b"Reference" in ref["generator"].tobytes()
