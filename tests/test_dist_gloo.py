"""World-size-2 gloo tests of the N>1 path (CPU): record-range ownership and the
compressed-blob gather that bench.py runs over RCCL on MI355X."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from pixiu_amd.dist import gather_blobs, record_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(rank)
    blob = torch.randint(0, 256, (1000 + 777 * rank,), dtype=torch.uint8, generator=g)
    out = gather_blobs(blob, dst=0)
    if rank == 0:
        exp = [torch.randint(0, 256, (1000 + 777 * r,), dtype=torch.uint8,
                             generator=torch.Generator().manual_seed(r)) for r in range(world)]
        q.put(all(torch.equal(a, b) for a, b in zip(out, exp)) and len(out) == world)
    else:
        q.put(out is None)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_blobs_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(res)


def test_record_range_partitions():
    for n in (0, 1, 7, 10_000, 10_001):
        for world in (1, 2, 3, 8):
            parts = [record_range(n, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            assert max(b - a for a, b in parts) - min(b - a for a, b in parts) <= 1


def _e2e_worker(rank, world, port, q):
    """One rank: encode its record range (the CPU oracle stands in for the GPU here),
    write a chunk blob, gather the blobs to rank 0 (gloo), and on rank 0 decode every
    record of every gathered blob back to its escaped doc."""
    import numpy as np
    import torch.distributed as dist
    from _oracle import EXACT, Oracle, assemble
    from pixiu_amd import blob, synth
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc = Oracle()
        cp = synth.make(2, 700)
        rps = 150
        a, b = record_range(cp.n, world, rank)
        chunks = []
        for s in range(a, b, rps):
            rows = range(s, min(b, s + rps))
            docs = [assemble(cp.key(i), cp.val(i)) for i in rows]
            comp, ch, _ = orc.encode_docs(docs)
            for c in sorted(set(ch)):
                sel = [k for k in range(len(docs)) if ch[k] == c]
                chunks.append(blob.Chunk(s // rps, c, [comp[k] for k in sel], [len(docs[k]) for k in sel],
                                         [False] * len(sel)))
        mine = torch.from_numpy(np.frombuffer(blob.write(chunks), np.uint8).copy())
        got = gather_blobs(mine, dst=0)
        if rank == 0:
            docs = [assemble(cp.key(i), cp.val(i)) for i in range(cp.n)]
            k = 0
            ok = len(got) == world
            for g in got:
                for c in blob.read(g.numpy().tobytes()):
                    for i in range(len(c.records)):
                        ok &= orc.decode_chunk(c.records, i, mode=EXACT) == docs[k]
                        k += 1
            q.put(ok and k == cp.n)
        else:
            q.put(got is None)
    finally:
        dist.destroy_process_group()


def test_sharded_encode_gather_decode_gloo():
    """The N>1 product path end to end on CPU: record-range shards per rank, chunk blobs
    (pixiu_amd/blob.py) gathered to rank 0, every record decodes from the gathered blobs."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_e2e_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(res)
