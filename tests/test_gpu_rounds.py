"""The reference's own shape at full size, and suffix-array rounds under their caps.

* config 3 as ONE store over all 10,000 pages (records_per_shard = 0: one PiXiuCtrl,
  chunks rotated by its MemPool rule, PiXiuCtrl.cpp:12-25): every chunk's first record,
  record count and sha256 of its compressed bytes equal tests/golden/c3_single.json,
  which the reference itself produced over the same 600 MB (tools/make_golden.py
  c3_single) -- ~52 chunks, so ~51 rotations, each checked;
* a batch whose suffix-array footprint exceeds the per-round position cap
  (PX_PSA_ROUND_MAX) runs in more rounds and gives the same bytes as one round and as
  the oracle;
* more shards than the first sort key's shard field holds (2^19) in one batch: split
  over rounds, every sampled record equals the oracle's one-record shard."""
import hashlib
import json
import os

import numpy as np
import pytest

from _oracle import Oracle, assemble

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c3_single.json")


def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def chunk_digest(res, comp):
    """per-chunk rows like tools/make_golden.chunk_digest"""
    chunks = {}
    for i, c in enumerate(res["chunk"].tolist()):
        chunks.setdefault(c, []).append(i)
    per = []
    for c in sorted(chunks):
        rows = chunks[c]
        per.append({"chunk": c, "first": rows[0], "records": len(rows),
                    "slots_in_order": [int(res["idx"][i]) for i in rows] == list(range(len(rows))),
                    "sha256": hashlib.sha256(b"".join(comp[i] for i in rows)).hexdigest()})
    return per


def test_config3_single_instance_matches_reference():
    _need_gpu()
    from pixiu_amd import synth
    g = json.load(open(GOLDEN))
    cp = synth.make(3, g["n"])
    assert hashlib.sha256(cp.keys.tobytes() + cp.vals.tobytes()).hexdigest() == g["input_sha256"]
    with px.Store(records_per_shard=0) as st:
        r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        assert int(r["status"].max()) == 0
        s = st.stats()
        assert (s["last_psa_shards"], s["last_walk_shards"]) == (1, 0)
        comp = st.export(px.records_of(r))
        got = chunk_digest(r, comp)
        assert all(c["slots_in_order"] for c in got)
        assert len(got) == len(g["chunks"])
        bad = [(a["chunk"], a["first"], b["first"], a["records"], b["records"])
               for a, b in zip(got, g["chunks"])
               if (a["first"], a["records"], a["sha256"]) != (b["first"], b["records"], b["sha256"])]
        assert not bad, f"{len(bad)} chunks differ from the reference, first: {bad[0]}"
        assert sum(map(len, comp)) == g["comp_bytes"]
        # a compat getitem sample spread over the chunks round-trips exactly
        sample = list(range(0, cp.n, 97))
        ex = st.get_batch([cp.key(i) for i in sample], px.EXACT)
        assert ex == [assemble(cp.key(i), cp.val(i)) for i in sample]


def _cap(v):
    old = os.environ.get("PX_PSA_ROUND_MAX")
    if v is None:
        os.environ.pop("PX_PSA_ROUND_MAX", None)
    else:
        os.environ["PX_PSA_ROUND_MAX"] = str(v)
    return old


@pytest.mark.parametrize("rps", [139, 0])
def test_round_cap_splits_the_batch(rps, store_factory, oracle):
    """config 3, 700 pages: with a cap of 20 M positions a round holds two 139-record
    shards (8.3 MB each); the single instance's window is cut to the cap"""
    from pixiu_amd import synth
    cp = synth.make(3, 700)
    kv = ((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    a = store_factory(records_per_shard=rps)
    ra = a.set_batch(*kv)
    rounds_a = a.stats()["last_psa_rounds"]
    old = _cap(20_000_000 if rps else 9_000_000)
    try:
        b = store_factory(records_per_shard=rps)
        rb = b.set_batch(*kv)
        rounds_b = b.stats()["last_psa_rounds"]
    finally:
        _cap(old)
    assert rounds_b > rounds_a
    assert int(rb["status"].max()) == 0
    assert rb["chunk"].tolist() == ra["chunk"].tolist() and rb["idx"].tolist() == ra["idx"].tolist()
    cb = b.export(px.records_of(rb))
    assert cb == a.export(px.records_of(ra))
    rows = list(range(139)) if rps else list(range(cp.n))
    oc, ochunk, oidx = oracle.encode_docs([assemble(cp.key(i), cp.val(i)) for i in rows])
    assert [cb[i] for i in rows] == oc
    assert rb["chunk"][rows].tolist() == ochunk and rb["idx"][rows].tolist() == oidx


def test_more_shards_than_one_round_holds(store_factory):
    """records_per_shard = 1 with 2^19 + 3,000 records: shard ids past the first sort
    key's 19-bit field go to a second round instead of aliasing"""
    n = (1 << 19) + 3000
    rng = np.random.default_rng(7)
    body = rng.integers(65, 69, size=(n, 24), dtype=np.uint8)  # repeats inside each record
    body[:, 12:] = body[:, :12]
    keys = [b"k%07d" % i for i in range(n)]
    kb = np.frombuffer(b"".join(keys), np.uint8).copy()
    ko = np.zeros(n + 1, np.uint64)
    np.cumsum([len(k) for k in keys], out=ko[1:])
    vb = body.reshape(-1).copy()
    vo = np.arange(n + 1, dtype=np.uint64) * 24
    st = store_factory(records_per_shard=1)
    r = st.set_batch((kb, ko), (vb, vo))
    assert int(r["status"].max()) == 0
    assert st.stats()["last_psa_rounds"] >= 2
    pick = sorted(set(np.linspace(0, n - 1, 400).astype(int).tolist()) | {(1 << 19) - 1, 1 << 19, n - 1})
    comp = st.export(px.records_of(r[pick]))
    orc = Oracle()
    for j, i in enumerate(pick):
        oc, ochunk, oidx = orc.encode_docs([assemble(keys[i], bytes(body[i]))])
        assert comp[j] == oc[0], i
        assert (int(r["chunk"][i]), int(r["idx"][i])) == (ochunk[0], oidx[0])
    got = st.get_batch([keys[i] for i in pick], px.EXACT)
    assert got == [assemble(keys[i], bytes(body[i])) for i in pick]
