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
    """Gather variable-size 1-D uint8 tensors to `dst`.  Returns the list of
    per-rank blobs on dst (trimmed to their true sizes), None elsewhere."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    rank = dist.get_rank()
    dev = blob.device
    size = torch.tensor([blob.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, size)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes) if sizes else 0
    padded = blob
    if blob.numel() < mx:
        padded = torch.zeros(mx, dtype=blob.dtype, device=dev)
        padded[:blob.numel()] = blob
    recv = [torch.empty(mx, dtype=blob.dtype, device=dev) for _ in range(world)] if rank == dst else None
    dist.gather(padded, recv, dst=dst)
    if rank != dst:
        return None
    return [r[:s] for r, s in zip(recv, sizes)]
