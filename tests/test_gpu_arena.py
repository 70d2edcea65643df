"""Record stores (px_runtime.cpp StoreArena): one reserved address range per context, mapped
on demand and reused after px_reset; `PX_NO_STORE_ARENA=1` puts them in heap slabs instead.
Both give the oracle's bytes and getitems, through resets and reloads."""
import pytest

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def _corpus(n=40):
    from pixiu_amd import synth
    cp = synth.make(3, n)
    return [cp.key(i) for i in range(cp.n)], [cp.val(i) for i in range(cp.n)]


@pytest.mark.parametrize("arena", [True, False])
def test_store_paths_match_oracle(store_factory, oracle, monkeypatch, arena):
    if not arena:
        monkeypatch.setenv("PX_NO_STORE_ARENA", "1")
    keys, vals = _corpus()
    want = oracle.run(keys, vals)
    st = store_factory(records_per_shard=0)
    for _ in range(3):  # (each reset reuses the store memory)
        st.reset()
        res = st.set_batch(keys, vals)
        assert st.export(px.records_of(res)) == want["comp"]
        assert st.get_batch(keys, px.COMPAT) == want["get"]
        assert st.stats()["last_get_device_keys"] == len(keys)
    blob = st.save()
    b = store_factory(records_per_shard=0)
    b.load(blob)
    assert b.get_batch(keys, px.COMPAT) == want["get"]
