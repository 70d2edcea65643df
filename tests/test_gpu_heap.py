"""The device heap reuses memory across batches of varying sizes (best-fit with
splitting and merging): the footprint after a sequence of differently sized batches
stays near the largest single batch's, and results stay exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def test_footprint_bounded_over_varying_batches(store_factory, oracle):
    from pixiu_amd import synth
    cp = synth.make(3, 400)
    st = store_factory(records_per_shard=64)
    held = []
    for n in (400, 130, 270, 64, 333, 200, 400, 97):
        st.reset()
        r = st.set_batch([cp.key(i) for i in range(n)], [cp.val(i) for i in range(n)])
        assert int(r["status"].max()) == 0
        held.append(st.stats()["device_bytes"])
        got = st.get_batch([cp.key(i) for i in range(0, n, 37)])
        assert all(g is not None for g in got)
    # the first 400-record batch sizes the heap; nothing after it needs more than a slab
    assert max(held) <= held[0] + (2 << 30), held
