"""Robustness of the set path: per-record results never
depend on scratch left by an earlier batch, a record that fails after the walk
placed it keeps its slot (later records of its chunk still succeed and may
reference it), and a single-shard batch far beyond 16 MB of escaped docs (the old
2^31 arena-offset limit) is bit-exact with the oracle."""
import os

import numpy as np
import pytest

from _oracle import assemble

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def _docs(cp, rows):
    return [assemble(cp.key(i), cp.val(i)) for i in rows]


@pytest.fixture
def env():
    saved = {}

    def setenv(k, v):
        saved.setdefault(k, os.environ.get(k))
        os.environ[k] = v

    yield setenv
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("rps", [0, 7])
def test_poisoned_scratch_between_batches(rps, store_factory, oracle, env):
    """Garbage in the batch scratch before every set batch (PX_DEBUG_POISON): batches of
    growing and shrinking sizes into one store give the oracle's bytes and placement."""
    from pixiu_amd import synth
    env("PX_DEBUG_POISON", "1")
    cp = synth.make(2, 400)
    st = store_factory(records_per_shard=rps)
    cuts = [0, 3, 90, 91, 250, 252, 400]
    res = []
    for a, b in zip(cuts, cuts[1:]):
        res.append(st.set_batch([cp.key(i) for i in range(a, b)], [cp.val(i) for i in range(a, b)]))
    r = np.concatenate(res)
    assert int(r["status"].max()) == 0
    comp = st.export(px.records_of(r))
    step = rps or cp.n
    want_get = []
    for s in range(0, cp.n, step):
        rows = list(range(s, min(cp.n, s + step)))
        w = oracle.run([cp.key(i) for i in rows], [cp.val(i) for i in rows])
        assert [comp[i] for i in rows] == w["comp"]
        assert r["chunk"][rows].tolist() == w["chunk"] and r["idx"][rows].tolist() == w["idx"]
        want_get += w["get"]
    assert st.get_batch([cp.key(i) for i in range(cp.n)]) == want_get


def test_failed_record_keeps_its_slot(store_factory, oracle, env):
    """A record failing after the walk placed it is registered dead: the chunk's slot
    numbering stays in step, later records succeed, and records referencing it decode."""
    from pixiu_amd import synth
    cp = synth.make(2, 60)
    keys, vals = [cp.key(i) for i in range(cp.n)], [cp.val(i) for i in range(cp.n)]
    st = store_factory(records_per_shard=0)
    env("PX_DEBUG_FAIL_REC", "17")
    r = st.set_batch(keys, vals, check=False)
    os.environ.pop("PX_DEBUG_FAIL_REC")
    assert int(r["status"][17]) == 4  # PX_ECORRUPT
    ok = [i for i in range(cp.n) if i != 17]
    assert int(r["status"][ok].max()) == 0
    assert r["idx"].tolist() == list(range(cp.n))  # slot 17 is taken by the failed record
    want = oracle.run(keys, vals)
    assert st.export(px.records_of(r[ok])) == [want["comp"][i] for i in ok]
    got = st.get_batch(keys)
    assert got[17] is None
    assert [got[i] for i in ok] == [want["get"][i] for i in ok]
    # the store keeps working after the failure: one more batch into the same chunk
    r2 = st.set_batch([b"after-" + keys[0]], [vals[0]])
    assert int(r2["status"][0]) == 0 and int(r2["idx"][0]) == cp.n


def test_single_shard_batch_beyond_16mb(store_factory, oracle):
    """rps = 0 and ~21 MB of escaped docs in one batch (crosses one pool rotation): node
    and hash sections are sized from the chunk bound, so every arena offset stays
    below 2^31; bytes and placement equal the oracle's single instance."""
    from pixiu_amd import synth
    n = 20_500
    cp = synth.make(2, n)
    st = store_factory(records_per_shard=0)
    r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    assert int(r["status"].max()) == 0
    assert int(r["chunk"].max()) >= 1
    oc, ochunk, oidx = oracle.encode_docs(_docs(cp, range(n)))
    assert st.export(px.records_of(r)) == oc
    assert r["chunk"].tolist() == ochunk and r["idx"].tolist() == oidx


@pytest.mark.parametrize("rps", [0, 64])
def test_device_inputs_with_offsets_not_starting_at_zero(rps, store_factory):
    """set_batch_device over a sub-range of device arrays (koff / voff start past 0, as
    the pieces of a batch split at kMaxBatchRaw do): every key is found again"""
    import torch
    from pixiu_amd import synth
    cp = synth.make(2, 600)
    kb = torch.from_numpy(cp.keys).cuda()
    ko = torch.from_numpy(cp.koff.astype(np.int64)).cuda()
    vb = torch.from_numpy(cp.vals).cuda()
    vo = torch.from_numpy(cp.voff.astype(np.int64)).cuda()
    st = store_factory(records_per_shard=rps)
    for a, b in ((0, 250), (250, 600)):
        r = st.set_batch_device(b - a, kb.data_ptr(), ko[a:].data_ptr(), vb.data_ptr(), vo[a:].data_ptr())
        assert int(r["status"].max()) == 0
    got = st.get_batch([cp.key(i) for i in range(cp.n)])
    assert got == [assemble(cp.key(i), cp.val(i)) for i in range(cp.n)]
