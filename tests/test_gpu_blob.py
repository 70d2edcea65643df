"""Chunk blob v1 through the HIP library: px_save -> px_load -> getitem round trips
(host and device buffers), the blob parses with pixiu_amd/blob.py and decodes with the
oracle, dead records stay dead, loaded stores keep accepting records (in a fresh
chunk), and two processes on one GPU gather their blobs to rank 0 (gloo), which
loads them and answers every key like the per-shard oracle."""
import os
import socket

import numpy as np
import pytest

from _oracle import EXACT, assemble

pytestmark = pytest.mark.gpu
px = pytest.importorskip("pixiu_amd")


def _cp(n=900):
    from pixiu_amd import synth
    return synth.make(2, n)


@pytest.mark.parametrize("rps", [0, 128])
def test_save_load_getitem(rps, store_factory, oracle):
    from pixiu_amd import blob
    cp = _cp()
    keys, vals = [cp.key(i) for i in range(cp.n)], [cp.val(i) for i in range(cp.n)]
    a = store_factory(records_per_shard=rps)
    r = a.set_batch(keys, vals)
    assert int(a.delete([keys[5], keys[400]]).max()) == 0
    b_host = a.save()
    # the blob is what blob.py reads: records in chunk-slot order, dead flags, decodable
    chunks = blob.read(b_host)
    assert sum(len(c.records) for c in chunks) == cp.n
    comp = a.export(px.records_of(r))
    flat = [(c, i) for c in chunks for i in range(len(c.records))]
    assert [c.records[i] for c, i in flat] == comp
    assert [c.dead[i] for c, i in flat] == [k in (5, 400) for k in range(cp.n)]
    for k in (0, 1, 399, cp.n - 1):
        c, i = flat[k]
        assert oracle.decode_chunk(c.records, i, mode=EXACT) == assemble(keys[k], vals[k])
    want = a.get_batch(keys)
    assert want[5] is None and want[400] is None
    # host blob -> fresh store
    b = store_factory(records_per_shard=rps)
    b.load(b_host)
    assert b.get_batch(keys) == want
    assert b.get_batch(keys, px.EXACT)[7] == assemble(keys[7], vals[7])
    assert list(b.contains([keys[5], keys[6]])) == [False, True]
    its = b.iter(b"rec/0000001")
    assert its is not None and len(its) == len(a.iter(b"rec/0000001"))
    # device blob -> fresh store
    import torch
    size = a.save_device(0, 0)
    dbuf = torch.empty(size, dtype=torch.uint8, device="cuda")
    a.save_device(dbuf.data_ptr(), size)
    assert dbuf.cpu().numpy().tobytes() == b_host
    c = store_factory(records_per_shard=rps)
    c.load(dbuf.data_ptr(), on_device=True, length=size)
    assert c.get_batch(keys) == want
    # a loaded store keeps accepting records; they land in a fresh chunk
    r2 = c.set_batch([b"new-key"], [b"new value " + vals[0][:50]])
    assert int(r2["status"][0]) == 0 and int(r2["idx"][0]) == 0
    assert c.get_batch([b"new-key"])[0] == assemble(b"new-key", b"new value " + vals[0][:50])
    assert int(c.delete([keys[9]])[0]) == 0 and c.get_batch([keys[9]])[0] is None


def test_load_rejects(store_factory):
    a = store_factory(records_per_shard=0)
    a.set_batch([b"k"], [b"v"])
    good = a.save()
    b = store_factory(records_per_shard=0)
    with pytest.raises(px.PxError):
        b.load(b"PXCB" + good[4:40])
    with pytest.raises(px.PxError):
        b.load(b"XXXX" + good[4:])
    with pytest.raises(px.PxError):  # a single-shard store must be empty to take a blob
        a.load(good)


def test_load_into_empty_single_shard(store_factory):
    """px_load into a single-shard store reports shard 0, the shard the chunks went into
    (include/pixiu_amd.h: *first_shard), whether the store is new or was reset."""
    cp = _cp(300)
    keys, vals = [cp.key(i) for i in range(cp.n)], [cp.val(i) for i in range(cp.n)]
    a = store_factory(records_per_shard=0)
    a.set_batch(keys, vals)
    blob_ = a.save()
    b = store_factory(records_per_shard=0)
    b.set_batch([b"tmp"], [b"x"])
    b.reset()
    assert b.load(blob_) == 0
    assert b.get_batch(keys) == a.get_batch(keys)
    c = store_factory(records_per_shard=0)
    assert c.load(blob_) == 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, rps, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pixiu_amd as px_
        from pixiu_amd.dist import gather_blobs, record_range
        cp = _cp(1000)
        a, b = record_range(cp.n, world, rank)
        with px_.Store(records_per_shard=rps) as st:
            r = st.set_batch([cp.key(i) for i in range(a, b)], [cp.val(i) for i in range(a, b)])
            ok = int(r["status"].max()) == 0
            mine = torch.from_numpy(np.frombuffer(st.save(), np.uint8).copy())
        got = gather_blobs(mine, dst=0)
        if rank != 0:
            q.put((rank, ok, None))
            return
        with px_.Store(records_per_shard=rps) as st0:
            for g in got:
                st0.load(g.numpy().tobytes())
            out = st0.get_batch([cp.key(i) for i in range(cp.n)])
        q.put((rank, ok, out))
    finally:
        dist.destroy_process_group()


def test_two_ranks_gather_and_load(oracle):
    """2 processes on device 0 (gloo): each stores its record range, saves a blob; rank 0
    gathers and loads both and answers every key like the oracle run per shard."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.multiprocessing as mp
    from pixiu_amd.dist import record_range
    world, rps = 2, 200
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, rps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((k, (ok, out)) for k, ok, out in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(60)
    assert all(ok for ok, _ in res.values())
    got = res[0][1]
    cp = _cp(1000)
    want = []
    for rank in range(world):
        a, b = record_range(cp.n, world, rank)
        for s in range(a, b, rps):
            rows = range(s, min(b, s + rps))
            want += oracle.run([cp.key(i) for i in rows], [cp.val(i) for i in rows])["get"]
    assert got == want
