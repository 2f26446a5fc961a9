"""Multi-GPU plumbing: reads shard round-robin over ranks (one process per GPU) with no data-path
collective; the only exchange is the final size/ratio reduction, done with
torch.distributed (RCCL over xGMI on MI355X, gloo in the CPU tests)."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    first_read: int   # global id of this rank's first read
    read_stride: int  # global ids: first_read + k * read_stride
    reads: int        # reads on this rank

    def global_ids(self):
        return [self.first_read + k * self.read_stride for k in range(self.reads)]


def shard_reads(reads_per_rank: int, rank: int, world: int) -> Shard:
    """Weak scaling: every rank owns `reads_per_rank` reads; global read r lives on rank r % world."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return Shard(rank, world, rank, world, reads_per_rank)


# counters reduced by SUM across ranks, in this order
COUNTERS = ("compressed_bytes", "samples", "errors", "chunks")


def reduce_run(counters: dict, elapsed_s: float, device=None) -> tuple[dict, float]:
    """All-reduce the per-rank counters (SUM) and the timed region (MAX)."""
    import torch
    import torch.distributed as dist

    vec = torch.tensor([int(counters.get(k, 0)) for k in COUNTERS], dtype=torch.int64, device=device)
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(vec, op=dist.ReduceOp.SUM)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return dict(zip(COUNTERS, (int(v) for v in vec.tolist()))), float(t.item())
