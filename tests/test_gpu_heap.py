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


@pytest.mark.parametrize("cfg,n,rps", [(3, 139, 139), (4, 40000, 8000), (4, 20000, 0)])
def test_memory_by_structure(cfg, n, rps, store_factory):
    """px_stats mem_*  account for the stored data: their sum is the heap's live
    bytes plus the mapped store range, less small control blocks; segment entries are kept only
    for records k_tokenize parses (none on these corpora), and the lane entries are what the
    records' tokens need (config 4: ~3 per record, not two per 251 byte)."""
    from pixiu_amd import synth
    cp = synth.make(cfg, n)
    st = store_factory(records_per_shard=rps)
    r = st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    assert int(r["status"].max()) == 0
    s = st.stats()
    mem = {k: int(v) for k, v in s.items() if k.startswith("mem_")}
    assert abs(sum(mem.values()) - int(s["device_live_bytes"])) < (1 << 20), (mem, s["device_live_bytes"])
    assert mem["mem_seg_bytes"] == 0
    assert mem["mem_comp_bytes"] >= int(s["comp_bytes"])
    if cfg == 4:
        assert mem["mem_lane_bytes"] < 16 * 8 * n, mem  # (round 5 reserved ~100 entries per record)
    got = st.get_batch([cp.key(i) for i in range(0, n, max(1, n // 50))])
    assert all(g is not None for g in got)
