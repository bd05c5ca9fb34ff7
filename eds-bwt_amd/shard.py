"""Pattern-batch sharding across GPUs.

The index is read-only and replicated on every GPU; patterns are independent, so
the batch is cut into contiguous pattern-id ranges, one per rank (one process per
GPU, torch.distributed).  The one exchange step: an all-gather of every rank's
(patterns, records), then the per-pattern counts and the 20-B occurrence records
gathered to rank 0 as tensors (RCCL over xGMI on GPUs; gloo on CPU).  Because the
ranges are contiguous, concatenation in rank order restores the reference's output
order (MOVE_EDSBWTSearch.cpp:111-136 processes patterns in file order).
"""
from __future__ import annotations

import numpy as np

REC_WORDS = 5  # edsbwt_occ = {pat, word, seg, word_in_seg, offset} (include/edsbwt.h)


def shard_range(npat: int, world: int, rank: int) -> tuple[int, int]:
    """[lo, hi) pattern indices of `rank`; pattern i is reported as #Pat = i + 1."""
    return npat * rank // world, npat * (rank + 1) // world


def shard_patterns(buf: np.ndarray, offs: np.ndarray, world: int, rank: int):
    """Slice a packed batch (bytes, offsets[npat+1]) to one rank's contiguous shard.
    Returns (bytes, offsets rebased to 0, first_pattern_id)."""
    lo, hi = shard_range(offs.size - 1, world, rank)
    b0, b1 = int(offs[lo]), int(offs[hi])
    return buf[b0:b1], (offs[lo:hi + 1] - offs[lo]).astype(np.uint64), lo + 1


def exchange_sizes(npat: int, nocc: int, device, group=None):
    """All-gather of every rank's (patterns, records): an int64 tensor [world, 2]."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    mine = torch.tensor([npat, nocc], dtype=torch.int64, device=device)
    out = torch.empty(world * 2, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, mine, group=group)
    return out.view(world, 2)


def _gather_padded(t, sizes: list[int], dst: int, group=None):
    """Gather 1-D tensors of per-rank lengths `sizes` to rank dst, padded to the longest
    (one collective; RCCL send/recv or gloo).  Returns the concatenation on dst, None elsewhere."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    m = max(max(sizes), 1)
    pad = torch.zeros(m, dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t
    outs = [torch.empty_like(pad) for _ in sizes] if rank == dst else None
    dist.gather(pad, outs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([o[:n] for o, n in zip(outs, sizes)])


def gather_counts(counts, sizes: list[int], dst: int = 0, group=None):
    """Every rank's per-pattern counts (tensor, any device) to rank dst in rank order."""
    return _gather_padded(counts, sizes, dst, group)


def gather_records(occ, sizes: list[int], dst: int = 0, group=None):
    """Every rank's occurrence records to rank dst in rank order.  `occ` is an int32/uint32
    tensor of n x 5 words (edsbwt_occ, e.g. a view of the engine's device records) or a
    numpy OCC array (moved to a CPU tensor); returns an n_total x 5 int32 tensor on dst."""
    import torch

    if isinstance(occ, np.ndarray):
        occ = torch.from_numpy(np.ascontiguousarray(occ).view(np.int32).reshape(-1))
    flat = occ.reshape(-1).view(torch.int32) if occ.dtype != torch.int32 else occ.reshape(-1)
    out = _gather_padded(flat, [n * REC_WORDS for n in sizes], dst, group)
    return None if out is None else out.view(-1, REC_WORDS)


def records_to_numpy(t) -> np.ndarray:
    """n x 5 int32 tensor -> numpy edsbwt_occ records."""
    from importlib import import_module

    occ_dtype = import_module("eds-bwt_amd").OCC_DTYPE
    a = t.detach().cpu().contiguous().numpy().astype(np.int32, copy=False)
    return a.view(np.uint32).view(occ_dtype).reshape(-1)
