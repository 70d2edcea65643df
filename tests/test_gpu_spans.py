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
