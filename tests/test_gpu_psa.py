"""The suffix-array setitem path (pixiu_amd/csrc/px_psa.hip) against the
GST walk it replaces and against the oracle:

* every BASELINE config: the same compressed bytes and placement with PX_PSA=0 (every
  shard walked by k_gst_encode) and with the default (shards encoded by PSA);
* a live chunk that outgrows the no-rotation bound in a later batch stays on PSA with
  the MemPool emulation: bytes equal the oracle's single instance;
* inputs on which the stale-pair check fires (small alphabets) still match the oracle.
"""
import os
import random

import numpy as np
import pytest

from _oracle import assemble

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def _run(cp, rps, psa, store_factory):
    old = os.environ.get("PX_PSA")
    os.environ["PX_PSA"] = "1" if psa else "0"
    try:
        st = store_factory(records_per_shard=rps)
        r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        stats = st.stats()
        comp = st.export(px.records_of(r))
        got = st.get_batch([cp.key(i) for i in range(0, cp.n, max(1, cp.n // 200))])
        return r, stats, comp, got
    finally:
        if old is None:
            os.environ.pop("PX_PSA", None)
        else:
            os.environ["PX_PSA"] = old


@pytest.mark.parametrize("cfg,n,rps", [(1, 1000, 0), (2, 3000, 500), (3, 60, 16), (4, 20000, 2000), (5, 48, 16)])
def test_psa_equals_walk(cfg, n, rps, store_factory):
    from pixiu_amd import synth
    cp = synth.make(cfg, n)
    ra, sa, ca, ga = _run(cp, rps, False, store_factory)
    rb, sb, cb, gb = _run(cp, rps, True, store_factory)
    assert sa["last_psa_shards"] == 0 and sb["last_psa_shards"] >= 1
    assert int(ra["status"].max()) == 0 and int(rb["status"].max()) == 0
    assert ca == cb
    assert ra["chunk"].tolist() == rb["chunk"].tolist() and ra["idx"].tolist() == rb["idx"].tolist()
    assert ga == gb


def test_psa_chunk_outgrows_bound_stays_psa(store_factory, oracle):
    """rps = 0: three batches; the third pushes the live chunk past kPsaMaxText, where the
    MemPool accounting is emulated on the suffix array (no walk, no replay); every record
    equals the oracle's single instance."""
    from pixiu_amd import synth
    cp = synth.make(2, 9000)
    st = store_factory(records_per_shard=0)
    res = []
    for a in (0, 3000, 6000):
        res.append(st.set_batch([cp.key(i) for i in range(a, a + 3000)], [cp.val(i) for i in range(a, a + 3000)]))
        s = st.stats()
        assert (s["last_psa_shards"], s["last_walk_shards"]) == (1, 0)
    r = np.concatenate(res)
    assert int(r["status"].max()) == 0
    oc, ochunk, oidx = oracle.encode_docs([assemble(cp.key(i), cp.val(i)) for i in range(cp.n)])
    assert st.export(px.records_of(r)) == oc
    assert r["chunk"].tolist() == ochunk and r["idx"].tolist() == oidx


def test_psa_small_alphabets_match_oracle(store_factory, oracle):
    """Random small-alphabet shards (where the reference's stale active-edge pair can
    change the output and the PSA check hands shards to the walk), batch of many shards."""
    rng = random.Random(20261016)
    keys, vals, groups = [], [], []
    seen = set()
    rps = 24
    for g in range(40):
        alpha = rng.choice([b"ab", b"abc", b"ABCDE", bytes([97, 98, 251]), bytes([251, 0, 2, 1, 97])])
        rows = []
        while len(rows) < rps:
            k = bytes(rng.choice(alpha) for _ in range(rng.randint(1, 10))) + b"%d" % g
            if k in seen:
                continue
            seen.add(k)
            rows.append(len(keys))
            keys.append(k)
            vals.append(bytes(rng.choice(alpha) for _ in range(rng.randint(0, 60))))
        groups.append(rows)
    st = store_factory(records_per_shard=rps)
    r = st.set_batch(keys, vals, check=False)
    s = st.stats()
    assert s["last_psa_shards"] + s["last_walk_shards"] == len(groups)
    comp = st.export(px.records_of(r[r["status"] == 0]))
    ok_rows = [i for i in range(len(keys)) if r["status"][i] == 0]
    pos = {i: k for k, i in enumerate(ok_rows)}
    for rows in groups:
        want = None
        try:
            want = oracle.run([keys[i] for i in rows], [vals[i] for i in rows], do_get=False)
        except RuntimeError:  # the reference would crash on this shard (PX_EREFCRASH here)
            assert any(int(r["status"][i]) != 0 for i in rows)
            continue
        assert [comp[pos[i]] for i in rows] == want["comp"]


def test_psa_long_runs_match_oracle(store_factory, oracle):
    """Runs of one byte longer than an ANSV workgroup (4,096 ranks): a run's suffixes lie at
    decreasing positions over consecutive ranks, so every rank of such a workgroup is one
    of its prefix minima and its queue of global searches (512) overflows to the owning
    waves (px_psa.hip k_psa_ansv_blk); bytes and placement equal the oracle's single
    instance."""
    keys = [b"run%d" % i for i in range(8)]
    vals = [b"a" * 20000, b"xyz" + b"a" * 9000 + b"q", b"b" * 5000 + b"a" * 5000, bytes(range(1, 251)) * 20,
            b"a" * 30000 + b"b", b"ab" * 6000, b"a" * 4097, b"\x00" * 12000]
    st = store_factory(records_per_shard=0)
    r = st.set_batch(keys, vals)
    s = st.stats()
    assert (s["last_psa_shards"], s["last_walk_shards"]) == (1, 0)
    assert int(r["status"].max()) == 0
    oc, ochunk, oidx = oracle.encode_docs([assemble(k, v) for k, v in zip(keys, vals)])
    assert st.export(px.records_of(r)) == oc
    assert r["chunk"].tolist() == ochunk and r["idx"].tolist() == oidx


def test_psa_slot_full_chunk_then_next_batch(store_factory, oracle):
    """A PSA live chunk filled to 65,535 docs: the next batch rotates at its first doc and
    stays on PSA (new chunk), bytes and placement equal the oracle's single instance."""
    from pixiu_amd import synth
    cp = synth.tiny_keys(70000)
    st = store_factory(records_per_shard=0)
    res = []
    for a, b in ((0, 65535), (65535, 70000)):
        res.append(st.set_batch([cp.key(i) for i in range(a, b)], [cp.val(i) for i in range(a, b)]))
        s = st.stats()
        assert (s["last_psa_shards"], s["last_walk_shards"]) == (1, 0)
    r = np.concatenate(res)
    assert int(r["status"].max()) == 0
    oc, ochunk, oidx = oracle.encode_docs([assemble(cp.key(i), cp.val(i)) for i in range(cp.n)])
    assert r["chunk"].tolist() == ochunk and r["idx"].tolist() == oidx
    assert st.export(px.records_of(r)) == oc


@pytest.mark.parametrize("cfg,n,rps", [(3, 128, 64), (5, 64, 32), (2, 4000, 1000)])
def test_segmented_sort_equals_radix(cfg, n, rps, store_factory):
    """The in-place segmented doubling sort (default) and the all-radix sort
    (PX_PSA_SEGSORT=0) give the same suffix array, hence the same bytes."""
    from pixiu_amd import synth
    cp = synth.make(cfg, n)
    out = []
    for seg in ("1", "0"):
        old = os.environ.get("PX_PSA_SEGSORT")
        os.environ["PX_PSA_SEGSORT"] = seg
        try:
            st = store_factory(records_per_shard=rps)
            r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
            assert int(r["status"].max()) == 0 and st.stats()["last_psa_shards"] >= 1
            out.append(st.export(px.records_of(r)))
        finally:
            if old is None:
                os.environ.pop("PX_PSA_SEGSORT", None)
            else:
                os.environ["PX_PSA_SEGSORT"] = old
    assert out[0] == out[1]


@pytest.mark.parametrize("syms", [5, 3, 4])
@pytest.mark.parametrize("cfg,n,rps", [(3, 64, 32), (5, 400, 200), (4, 20000, 0)])
def test_odd_pass_first_sort(syms, cfg, n, rps, store_factory, monkeypatch):
    """The first suffix sort with 5 / 3 passes (odd: its last pass used to read and write the
    same key buffer, px_route.h) and 4: the same bytes and placement as the default 6-symbol
    sort.  (5, 400, 200) is config 5 across MemPool rotations, the shape of round 5's second
    fault; (4, 20000, 0) the 251-heavy single instance."""
    from pixiu_amd import synth
    cp = synth.make(cfg, n)
    out = []
    for s in (None, str(syms)):
        if s is None:
            monkeypatch.delenv("PX_PSA_SYMS", raising=False)
        else:
            monkeypatch.setenv("PX_PSA_SYMS", s)
        st = store_factory(records_per_shard=rps)
        r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        assert int(r["status"].max()) == 0 and st.stats()["last_psa_shards"] >= 1
        out.append((st.export(px.records_of(r)), r["chunk"].tolist(), r["idx"].tolist()))
    assert out[0] == out[1]
