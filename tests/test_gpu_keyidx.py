"""The device key index (px_keyidx.hip): getitem batches whose keys it can answer resolve
on the GPU, every other batch on the host, with the same results either way -- checked
against the CPU oracle across replaces inside and across batches, deletes, missing keys,
exact mode and host / device output buffers."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def _ops(seed=3, n=3000, keyspace=900):
    rng = np.random.default_rng(seed)
    ks = [b"key/%05d" % int(rng.integers(keyspace)) for _ in range(n)]
    vs = [bytes(rng.choice(list(b"abcdefghij<>/=\xfb"), size=int(rng.integers(1, 400))).tolist()) for _ in range(n)]
    return ks, vs


def test_single_instance_matches_oracle(store_factory, oracle):
    ks, vs = _ops()
    st = store_factory(records_per_shard=0)
    sh = oracle.new()
    # three batches (replaces within and across them), then deletes
    for a, b in ((0, 1000), (1000, 2200), (2200, 3000)):
        st.set_batch(ks[a:b], vs[a:b])
        for k, v in zip(ks[a:b], vs[a:b]):
            sh.set(k, v)
    live = sorted(set(ks))
    got = st.get_batch(live)
    assert st.stats()["last_get_device_keys"] == len(live)  # every key on the device
    assert got == [sh.get(k) for k in live]
    assert st.get_batch(live, px.EXACT) == [sh.get(k, 1) for k in live]
    dels = live[::5]
    assert st.delete(dels).tolist() == [sh.delete(k) for k in dels]
    assert st.get_batch(live) == [sh.get(k) for k in live]  # (deleted keys: the host path)
    rest = [k for k in live if k not in set(dels)]
    assert st.get_batch(rest) == [sh.get(k) for k in rest]
    assert st.stats()["last_get_device_keys"] == len(rest)
    assert st.get_batch(rest + [b"nope"]) == [sh.get(k) for k in rest] + [None]
    assert st.stats()["last_get_device_keys"] == 0


def test_sharded_device_buffer_and_replaces(store_factory, oracle):
    """64-record shards, a key set again in a later shard (the older copy deleted from
    its shard): the device answers with the newest copy, as the host does"""
    import torch
    from pixiu_amd import synth
    cp = synth.make(2, 640)
    keys = [cp.key(i) for i in range(cp.n)]
    vals = [cp.val(i) for i in range(cp.n)]
    st = store_factory(records_per_shard=64)
    st.set_batch(keys, vals)
    again = keys[:50]
    newv = [v[::-1] for v in vals[:50]]
    st.set_batch(again, newv)
    dev = torch.device("cuda", 0)
    out = torch.empty(4 << 20, dtype=torch.uint8, device=dev)
    rc, off, ln, sts, _ = st.get_batch_device(keys, out.data_ptr(), out.numel(), px.COMPAT)
    assert rc == px.PX_OK and st.stats()["last_get_device_keys"] == len(keys)
    host = out.cpu().numpy()
    got = [host[int(o):int(o) + int(n)].tobytes() for o, n in zip(off, ln)]
    # the oracle per shard: the first 640 records in 10 shards, then the 50 new ones in shard 10
    want = {}
    for s0 in range(0, 640, 64):
        sh = oracle.new()
        for k, v in zip(keys[s0:s0 + 64], vals[s0:s0 + 64]):
            sh.set(k, v)
        for k in keys[s0:s0 + 64]:
            want[k] = sh.get(k)
    sh = oracle.new()
    for k, v in zip(again, newv):
        sh.set(k, v)
    for k in again:
        want[k] = sh.get(k)
    assert got == [want[k] for k in keys]
    assert st.get_batch(keys) == got


@pytest.mark.parametrize("rps", [0, 16])
def test_skipped_critbit_inserts(store_factory, oracle, rps):
    """Keys that extend another key by a 251 (the reference's CritBit skips their insert,
    CritBitTree.cpp:96-100: stored, but no walk reaches them): getitem / contains answer
    NULL / 0 for them like the reference, on the device path and the host path alike
    (the key map's hint must not shortcut the walk for them)."""
    import random
    rng = random.Random(251)
    keys, seen = [], set()
    while len(keys) < 160:
        k = bytes(rng.choice(b"ab\xfb") for _ in range(rng.randint(1, 5)))
        if k not in seen:
            seen.add(k)
            keys.append(k)
    vals = [bytes(rng.choice(b"xyz\xfb") for _ in range(rng.randint(0, 40))) for _ in keys]
    st = store_factory(records_per_shard=rps)
    st.set_batch(keys, vals)
    want = []
    step = rps or len(keys)
    for s0 in range(0, len(keys), step):
        sh = oracle.new()
        for k, v in zip(keys[s0:s0 + step], vals[s0:s0 + step]):
            sh.set(k, v)
        want += [sh.get(k) for k in keys[s0:s0 + step]]
    assert any(w is None for w in want)  # (the quirk is exercised)
    got = st.get_batch(keys)
    assert got == want
    assert st.contains(keys).tolist() == [w is not None for w in want]
    found = [k for k, w in zip(keys, want) if w is not None]
    assert st.get_batch(found) == [w for w in want if w is not None]


def test_pieces_keep_span_tables(store_factory):
    """A batch over 512 MB raw into one shard is stored in pieces; every record keeps its
    span table (its chunk's records stay within the span entries' 2 GiB reach: the record
    stores share one reserved address range) and every key resolves on the device, also
    after resets that reuse the memory (CHANGELOG.md round 4)."""
    import numpy as np
    import torch
    from pixiu_amd import synth
    cp = synth.make(3)
    dev = torch.device("cuda", 0)
    kb = torch.from_numpy(cp.keys).to(dev)
    ko = torch.from_numpy(cp.koff.astype(np.int64)).to(dev)
    vb = torch.from_numpy(cp.vals).to(dev)
    vo = torch.from_numpy(cp.voff.astype(np.int64)).to(dev)
    keys = (np.ascontiguousarray(cp.keys), cp.koff.astype(np.uint64))
    cap = int(2 * cp.raw_bytes + 256 * cp.n + (1 << 20))
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    st = store_factory(records_per_shard=0)
    first = None
    for _ in range(3):
        st.reset()
        st.set_batch_device(cp.n, kb.data_ptr(), ko.data_ptr(), vb.data_ptr(), vo.data_ptr(), check=True)
        rc, off, ln, sts, _ = st.get_batch_device(keys, out.data_ptr(), cap, px.COMPAT)
        assert rc == px.PX_OK
        s = st.stats()
        assert s["last_get_device_keys"] == cp.n and s["last_gather_queries"] == cp.n
        got = out[: int(off[-1]) + int(ln[-1])].cpu().numpy()
        h = hash(got.tobytes())
        first = h if first is None else first
        assert h == first


@pytest.mark.parametrize("rps", [0, 64])
def test_after_set_docs(store_factory, oracle, rps):
    """Records stored as ready docs (px_set_docs) have no device-index entry; they replace
    indexed records, so batches holding their keys go to the host path, batches of other keys
    stay on the device, and every answer equals the oracle fed the same records as setitem
    (a ready doc equal to assemble(k, v) stores what setitem(k, v) stores)."""
    import _oracle
    ks, vs = _ops(seed=11, n=600, keyspace=400)
    st = store_factory(records_per_shard=rps)
    st.set_batch(ks[:500], vs[:500])
    st.set_docs([_oracle.assemble(k, v) for k, v in zip(ks[500:], vs[500:])])
    # shards of rps records, each its own oracle instance; a key answers from the shard of
    # its newest copy (later shards win)
    step = rps or 600
    shards = []
    for s0 in range(0, 600, step):
        sh = oracle.new()
        for k, v in zip(ks[s0:s0 + step], vs[s0:s0 + step]):
            sh.set(k, v)
        shards.append(sh)
    newest = {k: i for i, k in enumerate(ks)}
    live = sorted(newest)
    want = {k: shards[newest[k] // step].get(k) for k in live}
    assert st.get_batch(live) == [want[k] for k in live]
    assert st.stats()["last_get_device_keys"] == 0  # (ready-doc keys: the host path)
    only_old = [k for k in live if k not in set(ks[500:])]
    assert st.get_batch(only_old) == [want[k] for k in only_old]
    assert st.stats()["last_get_device_keys"] == len(only_old)


def test_device_keys_and_results(store_factory):
    """px_get_batch_dev: keys and results in device memory.  Answered on the device it gives
    the host-key call's bytes, lengths and statuses; keys the index cannot answer (a missing
    key) go the host path and still land in the device arrays; too little room returns
    PX_ESPACE with the needed size."""
    import torch
    from pixiu_amd import synth
    cp = synth.make(4, 20000)
    st = store_factory(records_per_shard=2000)
    st.set_batch((cp.keys, cp.koff.astype(np.uint64)), (cp.vals, cp.voff.astype(np.uint64)))
    dev = torch.device("cuda", 0)
    keys = [cp.key(i) for i in range(0, cp.n, 3)]

    def run(ks, cap):
        kb, ko = px.csr(ks)
        dkb = torch.from_numpy(kb.copy() if kb.size else np.zeros(1, np.uint8)).to(dev)
        dko = torch.from_numpy(ko.astype(np.int64)).to(dev)
        n = len(ks)
        out = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
        off = torch.full((n,), 7, dtype=torch.int64, device=dev)
        ln = torch.full((n,), 7, dtype=torch.int32, device=dev)
        sts = torch.full((n,), 7, dtype=torch.int32, device=dev)
        rc, need = st.get_batch_dev(n, dkb.data_ptr(), dko.data_ptr(), out.data_ptr(), cap, off.data_ptr(),
                                    ln.data_ptr(), sts.data_ptr())
        return rc, need, out, off.cpu().numpy(), ln.cpu().numpy(), sts.cpu().numpy()

    want = st.get_batch(keys)
    rc, need, out, off, ln, sts = run(keys, 64 << 20)
    assert rc == px.PX_OK and st.stats()["last_get_device_keys"] == len(keys)
    h = out.cpu().numpy()
    assert (sts == 0).all()
    assert [h[o:o + l].tobytes() for o, l in zip(off, ln)] == want
    # a missing key: the host path, results still in the device arrays
    ks2 = keys[:100] + [b"no such key"] + keys[100:200]
    rc, need, out, off, ln, sts = run(ks2, 64 << 20)
    assert rc == px.PX_ENOTFOUND and st.stats()["last_get_device_keys"] == 0
    h = out.cpu().numpy()
    assert sts[100] == px.PX_ENOTFOUND and (np.delete(sts, 100) == 0).all()
    got = [None if s else h[o:o + l].tobytes() for o, l, s in zip(off, ln, sts)]
    assert got == st.get_batch(ks2)
    # too little room
    rc, need, *_ = run(keys, 4096)
    assert rc == px.PX_ESPACE and need > 4096


def test_big_batch_repeats_across_shards(store_factory, oracle):
    """A batch past the host-thread threshold (70,000 records, 2,000-record shards) whose keys
    repeat inside shards and across them, then a second such batch: the key map's partitions,
    the tries and the index entries take their parallel paths (set_batch runs the CritBit
    inserts on a helper thread); every key answers with its newest shard's value, as the
    per-shard oracle says"""
    import torch
    rng = np.random.default_rng(20261019)
    n, rps, space = 70000, 2000, 40000
    batches = []
    for _ in range(2):
        ks = [b"k%06d" % int(x) for x in rng.integers(space, size=n)]
        vs = [bytes(rng.integers(97, 123, size=int(rng.integers(20, 100))).astype(np.uint8)) for _ in range(n)]
        batches.append((ks, vs))
    st = store_factory(records_per_shard=rps)
    for ks, vs in batches:
        r = st.set_batch(ks, vs)
        assert int(r["status"].max()) == 0
    want = {}
    for ks, vs in batches:
        for s0 in range(0, n, rps):
            sh = oracle.new()
            for k, v in zip(ks[s0:s0 + rps], vs[s0:s0 + rps]):
                sh.set(k, v)
            for k in ks[s0:s0 + rps]:
                want[k] = sh.get(k)
    keys = sorted(want)
    dev = torch.device("cuda", 0)
    out = torch.empty(16 << 20, dtype=torch.uint8, device=dev)
    rc, off, ln, sts, _ = st.get_batch_device(keys, out.data_ptr(), out.numel(), px.COMPAT)
    assert rc == px.PX_OK
    host = out.cpu().numpy()
    got = [host[int(o):int(o) + int(m)].tobytes() for o, m in zip(off, ln)]
    assert got == [want[k] for k in keys]
    sample = keys[::97]
    assert st.get_batch(sample) == [want[k] for k in sample]
