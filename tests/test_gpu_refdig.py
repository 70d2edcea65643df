"""Full-size parity against the REFERENCE ITSELF: every record of every BASELINE config at
the bench's shard size (and config 3 as the reference's single instance), stored on the
GPU, read back through compat getitem, and compared with per-record digests of the
reference's own output on the same corpus and shards (tests/golden/refdig_*.npz, made by
tools/make_refdigests.py from oracle/_ref/libpxref.so in the build container).

Compared per record: the compat getitem drain (PiXiuCtrl::getitem + PXSGen,
PiXiuCtrl.cpp:59-61, PiXiuStr.h:129-198 -- the literal north-star contract, decoder bugs
included), the compressed bytes (SuffixTree.cpp:291-304 + PiXiuStr.cpp:16-118) and the
(chunk, slot) placement (PiXiuCtrl.cpp:13-25)."""
import numpy as np
import pytest

import _refdig

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")

CASES = [(2, 2000), (3, 139), (3, 0), (4, 8000), (5, 126)]


@pytest.mark.parametrize("cfg,rps", CASES, ids=[f"c{c}_rps{r}" for c, r in CASES])
def test_every_record_matches_reference_digests(cfg, rps):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ref = _refdig.load(cfg, rps)
    assert ref is not None, f"missing fixture {_refdig.path(cfg, rps)}"
    from pixiu_amd import synth
    cp = synth.make(cfg)
    assert cp.n == int(ref["n"])
    import hashlib
    assert hashlib.sha256(cp.keys.tobytes() + cp.vals.tobytes()).hexdigest().encode() == ref["input_sha256"].tobytes()
    dev = torch.device("cuda", 0)
    with px.Store(records_per_shard=rps) as st:
        res = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        assert int(res["status"].max()) == 0
        out, off, ln = _refdig.compat_all(st, (cp.keys, cp.koff.astype(np.uint64)), dev)
        r = _refdig.check_store(ref, st, res, out, off, ln)
    print(f"config {cfg} rps {rps}: {r}")
    assert r["placement_ne_reference"] == 0
    assert r["comp_ne_reference"] == 0
    assert r["compat_ne_reference"] == 0, r["first_bad"]
