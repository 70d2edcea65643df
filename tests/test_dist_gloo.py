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
