"""Pattern-batch sharding across GPUs.

The index is read-only and replicated on every GPU; patterns are independent, so
the batch is cut into contiguous pattern-id ranges, one per rank (one process per
GPU, torch.distributed).  The only exchange is the gather of the per-pattern
counts (and, optionally, the occurrence records) to rank 0 over RCCL; because the
ranges are contiguous, concatenation in rank order restores the reference's
output order (MOVE_EDSBWTSearch.cpp:111-136 processes patterns in file order).
"""
from __future__ import annotations

import numpy as np


def shard_range(npat: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) pattern indices of `rank`; pattern i is reported as #Pat = i + 1."""
    return npat * rank // world, npat * (rank + 1) // world


def shard_patterns(buf: np.ndarray, offs: np.ndarray, world: int, rank: int):
    """Slice a packed batch (bytes, offsets[npat+1]) to one rank's contiguous shard.
    Returns (bytes, offsets rebased to 0, first_pattern_id)."""
    lo, hi = shard_range(offs.size - 1, world, rank)
    b0, b1 = int(offs[lo]), int(offs[hi])
    return buf[b0:b1], (offs[lo:hi + 1] - offs[lo]).astype(np.uint64), lo + 1


def gather_counts(counts, world: int, npat_total: int, group=None):
    """All ranks' counts (torch tensors, any device; uneven shards allowed) gathered in
    rank order.  Uses all_gather over padded equal-size buffers (RCCL on GPU, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return counts
    size = -(-npat_total // world) + 1
    pad = torch.zeros(size, dtype=counts.dtype, device=counts.device)
    pad[: counts.numel()] = counts
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    parts = []
    for r in range(world):
        lo, hi = shard_range(npat_total, world, r)
        parts.append(outs[r][: hi - lo])
    return torch.cat(parts)


def gather_records(occ: np.ndarray, world: int, group=None) -> np.ndarray:
    """Concatenate every rank's occurrence records (numpy structured arrays) on all
    ranks, in rank order (object all-gather; records are host-side for CSV output)."""
    import torch.distributed as dist

    if world == 1:
        return occ
    outs = [None] * world
    dist.all_gather_object(outs, occ, group=group)
    return np.concatenate(outs)
