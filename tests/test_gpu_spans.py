"""Span tables: full-range getitem served by k_gather from each
record's compat expansion as literal runs, built at setitem by k_decode_addr +
k_span_build.  The gathered bytes must equal the segment walk's (PX_SPANS=0) and the
oracle's, in compat and exact mode, for every BASELINE config shape."""
import os

import numpy as np
import pytest

from _oracle import assemble

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def _with_spans(on, fn):
    old = os.environ.get("PX_SPANS")
    os.environ["PX_SPANS"] = "1" if on else "0"
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop("PX_SPANS", None)
        else:
            os.environ["PX_SPANS"] = old


@pytest.mark.parametrize("cfg,n,rps", [(1, 1000, 0), (2, 3000, 500), (3, 60, 16), (4, 20000, 2000), (5, 48, 16)])
def test_gather_equals_walk(cfg, n, rps, store_factory):
    from pixiu_amd import synth
    cp = synth.make(cfg, n)
    keys = [cp.key(i) for i in range(n)]

    def run():
        st = store_factory(records_per_shard=rps)
        r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        assert int(r["status"].max()) == 0
        g = st.get_batch(keys)
        s1 = st.stats()
        e = st.get_batch(keys, mode=px.EXACT)
        s2 = st.stats()
        recs = px.records_of(r)
        parts = st.parse_batch(recs[:: max(1, n // 50)])
        return g, e, parts, s1, s2

    g1, e1, p1, s1, s2 = _with_spans(True, run)
    g0, e0, p0, t1, t2 = _with_spans(False, run)
    assert s1["span_entries"] > 0 and t1["span_entries"] == 0
    # every record has a table unless its compat expansion overran doc + 64 bytes
    assert s1["last_gather_queries"] >= 0.9 * n and t1["last_gather_queries"] == 0
    assert s2["last_gather_queries"] > 0  # exact mode: records whose compat expansion is the doc
    assert g1 == g0 and e1 == e0 and p1 == p0
    # exact getitem is the original doc
    assert e1 == [assemble(cp.key(i), cp.val(i)) for i in range(n)]


def test_gather_matches_oracle_compat_bugs(store_factory, oracle):
    """Config 3 shards (compat != exact on some records): gathered compat bytes equal the
    oracle's PXSGen restatement record by record."""
    from pixiu_amd import synth
    cp = synth.make(3, 128)
    st = store_factory(records_per_shard=64)
    r = st.set_batch([cp.key(i) for i in range(128)], [cp.val(i) for i in range(128)])
    got = st.get_batch([cp.key(i) for i in range(128)])
    assert st.stats()["last_gather_queries"] >= 100
    want = []
    for a in (0, 64):
        want += oracle.run([cp.key(i) for i in range(a, a + 64)], [cp.val(i) for i in range(a, a + 64)])["get"]
    assert got == want
    assert int(r["status"].max()) == 0


def test_gather_capped_output(store_factory):
    """A device output buffer too small for the whole batch: PX_ESPACE with the needed
    size, then the full batch with room; gathered and walked bytes agree."""
    import torch
    from pixiu_amd import synth
    cp = synth.make(2, 500)
    keys = [cp.key(i) for i in range(500)]
    st = store_factory(records_per_shard=250)
    st.set_batch(keys, [cp.val(i) for i in range(500)])
    buf = torch.empty(1 << 12, dtype=torch.uint8, device="cuda")
    rc, off, ln, stt, need = st.get_batch_device(keys, buf.data_ptr(), buf.numel())
    assert rc == px.PX_ESPACE and need > buf.numel()
    buf = torch.empty(need, dtype=torch.uint8, device="cuda")
    rc, off, ln, stt, need2 = st.get_batch_device(keys, buf.data_ptr(), buf.numel())
    assert rc == px.PX_OK and (stt == 0).all()
    h = buf.cpu().numpy()
    got = [h[int(o):int(o) + int(l)].tobytes() for o, l in zip(off, ln)]
    assert got == st.get_batch(keys)


def test_exact_tables_near_length_251_aliases(store_factory):
    """Config 5 at the bench's shard size (126 records of 65,531 B): some records' streams
    hold a length-251 run token, which the decoder reads as an escape (the reference's alias,
    PiXiuStr.cpp:61-78), so their exact expansion is not their doc.  The exact span tables
    (built from 4 KB pieces, and whole for records whose pieces do not reassemble the doc)
    must serve what the walk decodes (PX_SPANS=0), record by record."""
    from pixiu_amd import synth
    n, rps = 252, 126
    cp = synth.make(5, n)
    keys = [cp.key(i) for i in range(n)]

    def run():
        st = store_factory(records_per_shard=rps)
        st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
        return st.get_batch(keys, mode=px.EXACT), st.get_batch(keys)

    e1, g1 = _with_spans(True, run)
    e0, g0 = _with_spans(False, run)
    assert g1 == g0
    assert e1 == e0
    docs = [assemble(cp.key(i), cp.val(i)) for i in range(n)]
    assert sum(e != d for e, d in zip(e1, docs)) < n  # (most exact expansions are their docs)


def _small_alphabet_docs(seed, n, lo, hi):
    """Docs over a few symbols with 251s and repeats of earlier material: self-referencing
    record tokens (the periodic case), 251 pairs at token edges, long nesting."""
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"ab<\xfb", np.uint8)
    keys, vals = [], []
    for i in range(n):
        L = int(rng.integers(lo, hi))
        v = alpha[rng.integers(0, len(alpha), L)].copy()
        for _ in range(int(rng.integers(1, 8))):  # copies of earlier parts, some overlapping
            a = int(rng.integers(0, L // 2))
            d = int(rng.integers(1, 64))
            m = int(rng.integers(16, L // 3))
            for k in range(m):
                if a + d + k < L:
                    v[a + d + k] = v[a + k]
        keys.append(b"k%05d" % i)
        vals.append(v.tobytes())
    return keys, vals


@pytest.mark.parametrize("rps", [0, 40])
def test_compat_tables_in_pieces(rps, store_factory):
    """Compat span tables decoded in 4 KB pieces cut at token starts (k_span_pieces) equal the
    whole-record decode (PX_SPAN_SPLIT=0) and the walk (PX_SPANS=0), compat and exact, on docs
    of 2-20 KB with self-referencing tokens and 251 runs."""
    keys, vals = _small_alphabet_docs(7 + rps, 120, 2000, 20000)

    def run():
        st = store_factory(records_per_shard=rps)
        r = st.set_batch(keys, vals)
        assert int(r["status"].max()) == 0
        g = st.get_batch(keys)
        gq = st.stats()["last_gather_queries"]
        return g, st.get_batch(keys, mode=px.EXACT), gq

    old = os.environ.get("PX_SPAN_SPLIT")
    try:
        os.environ["PX_SPAN_SPLIT"] = "1"
        g1, e1, q1 = _with_spans(True, run)
        os.environ["PX_SPAN_SPLIT"] = "0"
        g2, e2, q2 = _with_spans(True, run)
    finally:
        if old is None:
            os.environ.pop("PX_SPAN_SPLIT", None)
        else:
            os.environ["PX_SPAN_SPLIT"] = old
    g0, e0, _ = _with_spans(False, run)
    assert q1 == q2 and q1 >= 0.5 * len(keys)
    assert g1 == g2 == g0
    assert e1 == e2 == e0


def _chain_docs(seed, n, size):
    """Each doc is the previous one with one random byte inserted: the text around the latest
    insertions occurs only in the previous doc, so a record's tokens reference the record
    before it, whose range references the one before that — nesting as deep as the shard."""
    rng = np.random.default_rng(seed)
    v = rng.integers(0, 256, size, dtype=np.uint8)
    vals = [v.tobytes()]
    for _ in range(n - 1):
        v = np.insert(v, int(rng.integers(0, len(v) + 1)), np.uint8(rng.integers(0, 256)))
        vals.append(v.tobytes())
    return [b"c%04d" % i for i in range(n)], vals


def test_deep_reference_chains(store_factory, oracle):
    """Walks nested past the decoder's LDS lane stack (frames spilled to scratch) and past the
    spill (the serial frame machine): gathered and walked compat bytes equal the oracle's
    PXSGen restatement record by record, and exact getitem is the doc."""
    n, rps = 96, 48
    keys, vals = _chain_docs(11, n, 1500)

    def run():
        st = store_factory(records_per_shard=rps)
        r = st.set_batch(keys, vals)
        assert int(r["status"].max()) == 0
        return st.get_batch(keys), st.get_batch(keys, mode=px.EXACT)

    g1, e1 = _with_spans(True, run)
    g0, e0 = _with_spans(False, run)
    want = []
    for a in range(0, n, rps):
        want += oracle.run(keys[a:a + rps], vals[a:a + rps])["get"]
    assert g1 == g0 == want
    docs = [assemble(k, v) for k, v in zip(keys, vals)]
    assert e1 == e0 == docs
