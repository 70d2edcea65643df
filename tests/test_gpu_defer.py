"""The write-behind queue of one-record setitem calls (px_opts.defer_bytes, px_flush;
include/pixiu_amd.h): the same calls with and without the queue return the same
`replaced` values and store the same bytes in the same slots, reads flush first, and
the reference's rotation by slot count (65,535 docs, PiXiuCtrl.cpp:13) lands where the
oracle puts it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def _calls(n, seed=5, keyspace=None):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = b"u/%06d" % (rng.integers(keyspace) if keyspace else i)
        v = bytes(rng.choice(list(b"abcdefgh<>/=\xfb"), size=int(rng.integers(0, 300))).tolist())
        out.append((k, v))
    return out


def test_defer_matches_one_call_per_record(store_factory, oracle):
    calls = _calls(2500, keyspace=1800)  # repeated keys: replaces inside and across flushes
    a = store_factory(records_per_shard=0, defer_bytes=64 << 10)
    b = store_factory(records_per_shard=0)
    ra, rb = [], []
    for k, v in calls:
        ra.append(a.set_batch([k], [v])[0])
        rb.append(b.set_batch([k], [v])[0])
    assert [int(x["replaced"]) for x in ra] == [int(x["replaced"]) for x in rb]
    assert all(int(x["chunk"]) == px.PX_PENDING for x in ra if int(x["status"]) == 0)
    last = a.flush()[0]
    assert int(last["chunk"]) == int(rb[-1]["chunk"]) and int(last["idx"]) == int(rb[-1]["idx"])
    sa, sb = a.stats(), b.stats()
    assert sa["deferred_records"] == 2500 and sa["deferred_mismatch"] == 0 and sa["deferred_flushes"] > 1
    assert sa["records"] == sb["records"] and sa["comp_bytes"] == sb["comp_bytes"]
    keys = sorted({k for k, _ in calls})
    la, _ = a.locate(keys)
    lb, _ = b.locate(keys)
    assert (la == lb).all()
    assert a.export(la) == b.export(lb)
    assert a.get_batch(keys) == b.get_batch(keys)
    # and both equal the oracle fed the same calls
    sh = oracle.new()
    want_rep = [sh.set(k, v)[0] for k, v in calls]
    assert want_rep == [int(x["replaced"]) for x in rb]
    assert a.get_batch(keys) == [sh.get(k) for k in keys]


def test_defer_reads_flush_first(store_factory):
    a = store_factory(records_per_shard=0, defer_bytes=1 << 30)
    a.set_batch([b"k1"], [b"v1"])
    assert a.contains([b"k1"]).tolist() == [True]  # contains flushes
    a.set_batch([b"k2"], [b"v2"])
    assert a.get_batch([b"k2"]) == [b"k2\xfb\x00v2\xfb\x02"]
    a.set_batch([b"k3"], [b"v3"])
    assert a.delete([b"k3"]).tolist() == [0]
    a.set_batch([b"k4"], [b"v4"])
    assert a.stats()["records"] == 4
    a.set_batch([b"k5"], [b"v5"])
    a.reset()  # drops the queue, like free_prop
    assert a.stats()["records"] == 0 and a.get_batch([b"k5"]) == [None]
    # an invalid record is refused at call time and never queued
    r = a.set_batch([b""], [b"x"], check=False)
    assert int(r[0]["status"]) == px.PX_EINVAL
    assert a.stats()["records"] == 0


def test_defer_slot_rotation_matches_oracle(store_factory, oracle):
    """66,000 key-only one-record calls: the 65,535-slot rotation inside the queue"""
    from pixiu_amd import synth
    cp = synth.tiny_keys(66000)
    a = store_factory(records_per_shard=0, defer_bytes=1 << 20)
    for i in range(cp.n):
        a.set_batch([cp.key(i)])
    a.flush()
    ref = oracle.run([cp.key(i) for i in range(cp.n)], [b""] * cp.n, do_get=False)
    keys = [cp.key(i) for i in range(cp.n)]
    recs, st = a.locate(keys)
    assert (st == 0).all()
    assert recs["chunk"].tolist() == ref["chunk"] and recs["idx"].tolist() == ref["idx"]
    assert a.export(recs[::97]) == ref["comp"][::97]


def test_failed_flush_is_reported(store_factory, monkeypatch):
    """A queued record whose flush fails (here: PX_DEBUG_SET_THROW makes the batch throw
    bad_alloc) is not silently lost: the read that triggered the flush fails, and a later
    px_flush still reports the failure once (flush_queue emptied the queue
    before the store and dropped the error)."""
    st = store_factory(records_per_shard=0, defer_bytes=1 << 20)
    r = st.set_batch([b"k/1"], [b"v" * 100])
    assert int(r["status"][0]) == 0 and int(r["chunk"][0]) == px.PX_PENDING
    monkeypatch.setenv("PX_DEBUG_SET_THROW", "1")
    with pytest.raises(px.PxError) as e:  # a read flushes first: the batch fails
        st.contains([b"k/1"])
    assert e.value.code == px.PX_ENOMEM
    monkeypatch.delenv("PX_DEBUG_SET_THROW")
    with pytest.raises(px.PxError) as e:  # ... and px_flush reports it afterwards
        st.flush()
    assert e.value.code == px.PX_ENOMEM
    st.flush()  # reported once
    assert not st.contains([b"k/1"])[0]
    # the store keeps working
    st.set_batch([b"k/2"], [b"w" * 50])
    assert st.get_batch([b"k/2"])[0] is not None
