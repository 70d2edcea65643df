"""Chunk rotation on the suffix-array path (px_psa.hip k_pool_*).

The reference rotates its live chunk before a doc once 2,048 MemPool pools are open
(PiXiuCtrl.cpp:13); the pool count follows the leaves and inner nodes its suffix tree
creates (MemPool.cpp:7-37, SuffixTree.cpp:148-227).  The suffix-array path emulates that
accounting and encodes shards of any size in rounds (one chunk window per round).  These
tests compare it with the oracle's single instance (chunk numbers, slots and compressed
bytes of every record) on shards that rotate, within one batch and across batches.  The reference's own rotation fixtures
(tests/golden/rotation.json, test_gpu_golden.py) take the same path.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from _oracle import Oracle, assemble

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def _oracle_shards(cp, rps):
    """oracle encode_docs per shard of rps records (rps = 0: one shard), on threads"""
    n = cp.n
    bounds = [(a, min(n, a + rps)) for a in range(0, n, rps)] if rps else [(0, n)]

    def one(ab):
        a, b = ab
        return Oracle().encode_docs([assemble(cp.key(i), cp.val(i)) for i in range(a, b)])

    with ThreadPoolExecutor(min(8, len(bounds))) as ex:
        parts = list(ex.map(one, bounds))
    comp, chunk, idx = [], [], []
    for c, ch, ix in parts:
        comp += c
        chunk += ch
        idx += ix
    return comp, chunk, idx


def _set(st, cp, pieces):
    res = []
    for a, b in pieces:
        res.append(st.set_batch([cp.key(i) for i in range(a, b)], [cp.val(i) for i in range(a, b)]))
    return np.concatenate(res)


@pytest.mark.parametrize("chain", [False, True])
def test_single_instance_rotates_like_the_oracle(chain, store_factory, monkeypatch):
    """config 3, 420 records (25 MB) in one batch at rps = 0: two rotations by pool count.
    chain: PX_DEBUG_POOL_CHAIN=1 skips the bound test, so every window runs the boundary
    chain; both must place every record where the reference does"""
    from pixiu_amd import synth
    if chain:
        monkeypatch.setenv("PX_DEBUG_POOL_CHAIN", "1")
    cp = synth.make(3, 420)
    st = store_factory(records_per_shard=0)
    r = _set(st, cp, [(0, cp.n)])
    s = st.stats()
    assert (s["last_psa_shards"], s["last_walk_shards"]) == (1, 0)
    assert s["last_psa_rotations"] >= 1 and s["last_psa_rounds"] >= 2
    assert int(r["status"].max()) == 0
    oc, ochunk, oidx = _oracle_shards(cp, 0)
    assert r["chunk"].tolist() == ochunk and r["idx"].tolist() == oidx
    assert max(ochunk) >= 1
    assert st.export(px.records_of(r)) == oc
    sample = list(range(0, cp.n, 7))
    assert st.parse_batch(px.records_of(r[sample]), px.EXACT) == [assemble(cp.key(i), cp.val(i)) for i in sample]


def test_rotation_across_batches_and_shards(store_factory):
    """config 3, two 300-record shards fed in 4 batches of 150: rotations fall inside
    batches and the live chunk is carried across batch boundaries"""
    from pixiu_amd import synth
    cp = synth.make(3, 600)
    st = store_factory(records_per_shard=300)
    r = _set(st, cp, [(0, 150), (150, 300), (300, 450), (450, 600)])
    assert int(r["status"].max()) == 0
    oc, ochunk, oidx = _oracle_shards(cp, 300)
    assert r["chunk"].tolist() == ochunk and r["idx"].tolist() == oidx
    assert max(ochunk) >= 1
    assert st.export(px.records_of(r)) == oc
    got = st.get_batch([cp.key(i) for i in range(0, cp.n, 5)])
    want = _oracle_get(cp, 300, range(0, cp.n, 5))
    assert got == want


def _oracle_get(cp, rps, rows):
    out = {}
    for a in range(0, cp.n, rps):
        want = [i for i in rows if a <= i < a + rps]
        if not want:
            continue
        o = Oracle().run([cp.key(i) for i in range(a, a + rps)], [cp.val(i) for i in range(a, a + rps)])
        for i in want:
            out[i] = o["get"][i - a]
    return [out[i] for i in rows]


@pytest.mark.parametrize("cfg,n,rps,chain", [(2, 20000, 0, False), (4, 60000, 0, False), (5, 400, 200, False),
                                             (4, 60000, 0, True)])
def test_pool_emulation_matches_oracle(cfg, n, rps, chain, store_factory, monkeypatch):
    """configs 2 / 4 (byte-251 stress) / 5: every record's chunk, slot and bytes (chain: the
    boundary chain in every window, as above)"""
    from pixiu_amd import synth
    if chain:
        monkeypatch.setenv("PX_DEBUG_POOL_CHAIN", "1")
    cp = synth.make(cfg, n)
    st = store_factory(records_per_shard=rps)
    r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    assert int(r["status"].max()) == 0
    oc, ochunk, oidx = _oracle_shards(cp, rps)
    assert r["chunk"].tolist() == ochunk and r["idx"].tolist() == oidx
    assert max(ochunk) >= 1
    assert st.export(px.records_of(r)) == oc


def _flag_round(k):
    old = os.environ.get("PX_DEBUG_PSA_FLAG_ROUND")
    os.environ["PX_DEBUG_PSA_FLAG_ROUND"] = str(k)
    return old


def _unflag(old):
    if old is None:
        os.environ.pop("PX_DEBUG_PSA_FLAG_ROUND", None)
    else:
        os.environ["PX_DEBUG_PSA_FLAG_ROUND"] = old


def test_walk_takes_over_after_a_rotation(store_factory):
    """The stale-pair check firing in the round after a rotation (test hook): the walk
    takes the shard's remaining docs in the new chunk, whose text starts past the closed
    chunk's in the arena; every record equals the oracle's single instance"""
    from pixiu_amd import synth
    cp = synth.make(3, 230)
    st = store_factory(records_per_shard=0)
    old = _flag_round(2)
    try:
        r = _set(st, cp, [(0, cp.n)])
    finally:
        _unflag(old)
    s = st.stats()
    assert s["last_walk_shards"] == 1 and s["last_psa_rotations"] >= 1
    assert int(r["status"].max()) == 0
    oc, ochunk, oidx = _oracle_shards(cp, 0)
    assert r["chunk"].tolist() == ochunk and r["idx"].tolist() == oidx
    assert st.export(px.records_of(r)) == oc


def test_walk_replays_the_live_chunk(store_factory):
    """The check firing on a batch whose live chunk came from an earlier batch (test
    hook): the walk replays the live chunk's docs, then continues; later batches go on
    from the walked tree"""
    from pixiu_amd import synth
    cp = synth.make(2, 3600)
    st = store_factory(records_per_shard=0)
    r1 = _set(st, cp, [(0, 2000)])
    old = _flag_round(1)
    try:
        r2 = _set(st, cp, [(2000, 3000)])
    finally:
        _unflag(old)
    assert st.stats()["last_walk_shards"] == 1
    r3 = _set(st, cp, [(3000, 3600)])
    r = np.concatenate([r1, r2, r3])
    assert int(r["status"].max()) == 0
    oc, ochunk, oidx = _oracle_shards(cp, 0)
    assert r["chunk"].tolist() == ochunk and r["idx"].tolist() == oidx
    assert st.export(px.records_of(r)) == oc
    got = st.get_batch([cp.key(i) for i in range(0, cp.n, 9)])
    assert got == [assemble(cp.key(i), cp.val(i)) for i in range(0, cp.n, 9)]
