"""BASELINE.json full sizes.

* config 3 at the benchmarked shard size: EVERY shard's compressed bytes and
  placement against the CPU oracle (one oracle instance per shard, on host threads),
  plus the compat getitem of a 1,000-record sample against the oracle's getitem;
* configs 2, 4 and 5 at their full record counts: every record's exact expansion
  equals its escaped doc (round trip), compat equals exact except where the
  reference's decoder bug hits (counted), and sampled whole shards are bit-exact
  with the oracle."""
import concurrent.futures as cf
import os

import numpy as np
import pytest

from _oracle import assemble

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")
THREADS = min(16, os.cpu_count() or 1)


def _docs(cp, rows):
    return [assemble(cp.key(i), cp.val(i)) for i in rows]


def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _store_all(st, cp):
    r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    assert int(r["status"].max()) == 0
    return r


def test_config3_every_shard_at_bench_rps(oracle):
    """All 10,000 pages at the bench's records_per_shard: every shard vs the oracle."""
    _need_gpu()
    from pixiu_amd import synth
    import bench
    rps = bench.DEFAULT_RPS[3]
    cp = synth.make(3)
    n = cp.n
    with px.Store(records_per_shard=rps) as st:
        r = _store_all(st, cp)
        comp = st.export(px.records_of(r))
        groups = [list(range(s, min(n, s + rps))) for s in range(0, n, rps)]
        with cf.ThreadPoolExecutor(THREADS) as ex:
            want = list(ex.map(lambda g: oracle.encode_docs(_docs(cp, g)), groups))
        bad = 0
        for g, (oc, ochunk, oidx) in zip(groups, want):
            bad += [comp[i] for i in g] != oc
            bad += r["chunk"][g].tolist() != ochunk or r["idx"][g].tolist() != oidx
        assert bad == 0, f"{bad} of {len(groups)} shards differ from the oracle"
        # compat getitem of the first 1,000 records against the oracle's getitem
        sample = [g for g in groups if g[0] < 1000]
        with cf.ThreadPoolExecutor(THREADS) as ex:
            gets = list(ex.map(lambda g: oracle.run([cp.key(i) for i in g], [cp.val(i) for i in g])["get"], sample))
        rows = [i for g in sample for i in g]
        assert st.get_batch([cp.key(i) for i in rows], px.COMPAT) == [x for gg in gets for x in gg]


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_full_size_round_trip(cfg, oracle):
    _need_gpu()
    from pixiu_amd import synth
    import bench
    rps = bench.DEFAULT_RPS[cfg]
    cp = synth.make(cfg)
    n = cp.n
    with px.Store(records_per_shard=rps) as st:
        r = _store_all(st, cp)
        recs = px.records_of(r)
        comp_all = st.export(recs)
        # chunks holding a len-251 alias record (251,251 + record fields): the only lossy case
        alias_chunks = {(int(r["shard"][i]), int(r["chunk"][i])) for i in range(n) if b"\xfb\xfb" in comp_all[i]}
        bad_exact = compat_diff = 0
        step = 4000
        for a in range(0, n, step):
            rows = range(a, min(n, a + step))
            ex = st.parse_batch(recs[a:a + len(rows)], px.EXACT)
            co = st.parse_batch(recs[a:a + len(rows)], px.COMPAT)
            for i, (e, c, d) in enumerate(zip(ex, co, _docs(cp, rows))):
                if e != d:
                    bad_exact += 1
                    assert (int(r["shard"][a + i]), int(r["chunk"][a + i])) in alias_chunks
                compat_diff += c != e
        print(f"config {cfg}: {n} records, exact != doc: {bad_exact}, compat != exact: {compat_diff}")
        # oracle sample: whole shards, compressed bytes and placement
        shards = (n + rps - 1) // rps
        picks = sorted(set(np.linspace(0, shards - 1, 4).astype(int).tolist()))
        groups = [list(range(s * rps, min(n, (s + 1) * rps))) for s in picks]
        with cf.ThreadPoolExecutor(THREADS) as ex:
            want = list(ex.map(lambda g: oracle.encode_docs(_docs(cp, g)), groups))
        for g, (oc, ochunk, oidx) in zip(groups, want):
            assert [comp_all[i] for i in g] == oc
            assert r["chunk"][g].tolist() == ochunk and r["idx"][g].tolist() == oidx
