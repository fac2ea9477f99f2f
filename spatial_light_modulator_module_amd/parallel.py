"""Batch sharding for one-process-per-GPU runs.

Holograms are independent, so a batch of B targets is split
into contiguous shards, one per rank, with no data-path collective; only the
final phase arrays travel, gathered to rank 0 (RCCL send/recv over xGMI in
libslm_hip, slm_plan_gather_phase). The same shard arithmetic drives bench.py,
the sequence CLI and the CPU (gloo) tests of the N > 1 path.
"""
from __future__ import annotations

import os


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_counts(total: int, nranks: int) -> list[int]:
    """Contiguous shard sizes: the first total % nranks ranks take one more."""
    if nranks < 1 or total < 0:
        raise ValueError("need nranks >= 1 and total >= 0")
    q, r = divmod(total, nranks)
    return [q + (1 if k < r else 0) for k in range(nranks)]


def shard_range(total: int, nranks: int, rank: int) -> range:
    """Indices of the holograms owned by `rank`."""
    counts = shard_counts(total, nranks)
    start = sum(counts[:rank])
    return range(start, start + counts[rank])


def assemble(parts: list, counts: list[int]):
    """Concatenate per-rank results (rank order) into the global batch order;
    the host-side twin of the RCCL gather, used by the gloo tests."""
    import numpy as np

    if len(parts) != len(counts):
        raise ValueError("one part per rank")
    for p, c in zip(parts, counts):
        if len(p) != c:
            raise ValueError(f"part of {len(p)} holograms where {c} were expected")
    return np.concatenate([np.asarray(p) for p in parts if len(p)], axis=0)
