"""Multi-GPU plumbing: one process per GPU, record ranges sharded across ranks
with no cross-GPU references; the only exchange is gathering every rank's
packed compressed blob to one rank (RCCL over xGMI on MI355X, gloo on CPU)."""
from __future__ import annotations


def record_range(n: int, world: int, rank: int) -> tuple:
    """Contiguous [a, b) of n records owned by `rank` (balanced, order-preserving)."""
    per, extra = divmod(n, world)
    a = rank * per + min(rank, extra)
    return a, a + per + (1 if rank < extra else 0)


def gather_blobs(blob, dst: int = 0):
    """Gather variable-size 1-D uint8 tensors to `dst`: the sizes by one all_gather, then
    every blob at its exact size, point to point (one batched group of sends / receives:
    grouped ncclSend / ncclRecv over xGMI with RCCL; plain isend / irecv with gloo, whose
    tensors live on the CPU).  Returns the list of per-rank blobs on dst (its own is the
    tensor passed in), None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = blob.device
    size = torch.tensor([blob.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, size)
    sizes = [int(s.item()) for s in sizes]
    out = None
    if rank == dst:
        out = [blob if r == dst else torch.empty(sizes[r], dtype=blob.dtype, device=dev) for r in range(world)]
        ops = [(dist.irecv, out[r], r) for r in range(world) if r != dst and sizes[r]]
    else:
        ops = [(dist.isend, blob, dst)] if blob.numel() else []
    if ops:
        if dist.get_backend() == "nccl":
            reqs = dist.batch_isend_irecv([dist.P2POp(f, t, peer) for f, t, peer in ops])
        else:
            reqs = [f(t, peer) for f, t, peer in ops]
        for q in reqs:
            q.wait()
    return out
