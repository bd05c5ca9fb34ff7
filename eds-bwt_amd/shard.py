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


class SizesExchange:
    """The per-step all-gather of every rank's (patterns, records) — each rank's offsets in the
    output — without a host round trip: the two numbers go up through a small ring of page-locked
    slots (no pageable copy, no synchronisation), the all-gather is asynchronous, and its result
    stays on the device until result() (outside the timed steps)."""

    RING = 4

    def __init__(self, device, group=None):
        import torch
        import torch.distributed as dist

        self.group = group
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        pin = self.device.type == "cuda"
        self.host = [torch.zeros(2, dtype=torch.int64, pin_memory=pin) for _ in range(self.RING)]
        self.mine = [torch.zeros(2, dtype=torch.int64, device=self.device) for _ in range(self.RING)]
        self.out = torch.zeros(self.world * 2, dtype=torch.int64, device=self.device)
        self.k = 0
        self.work = None
        self.ev = [None] * self.RING

    def start(self, npat: int, nocc: int, async_op: bool = True):
        import torch
        import torch.distributed as dist

        k = self.k % self.RING
        self.k += 1
        if self.ev[k] is not None:
            self.ev[k].synchronize()  # the copy out of this slot RING steps ago (long done)
        self.host[k][0], self.host[k][1] = int(npat), int(nocc)
        if self.device.type == "cuda":
            self.mine[k].copy_(self.host[k], non_blocking=True)
            self.ev[k] = torch.cuda.Event()
            self.ev[k].record()
        else:
            self.mine[k].copy_(self.host[k])
        if self.work is not None:
            self.work.wait()
        self.work = dist.all_gather_into_tensor(self.out, self.mine[k], group=self.group, async_op=async_op)
        return self.work

    def result(self):
        """[world, 2] int64 (patterns, records) per rank, of the last start()."""
        if self.work is not None:
            self.work.wait()
            self.work = None
        return self.out.view(self.world, 2)


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


class CountsGather:
    """The per-step counts gather of one batch shape, set up once.  Every rank's
    shard size follows from the static contiguous split (`sizes`, the same on every rank), so a
    step neither reads sizes back to the host nor allocates: rank dst holds one [sum(sizes)]
    output tensor and, when the shards are equal (C3: 10M per GPU, C4: 100M / N), receives every
    rank's counts straight into its slice of it (rank order = the file's line order, no copy, no
    cat).  Unequal shards go through a preallocated padded send buffer and padded receive slots,
    compacted by result().  start() returns the collective's work handle when async_op (the
    caller keeps the source tensor unchanged until wait(): bench.py alternates two count
    buffers, so the gather of step i overlaps the search of step i + 1)."""

    def __init__(self, sizes, device, dtype=None, dst: int = 0, group=None):
        import torch
        import torch.distributed as dist

        self.sizes = [int(x) for x in sizes]
        self.dst, self.group = dst, group
        self.rank = dist.get_rank(group)
        self.m = max(max(self.sizes), 1)
        self.equal = all(n == self.m for n in self.sizes)
        dtype = dtype or torch.int32
        self.pad = None if self.equal else torch.zeros(self.m, dtype=dtype, device=device)
        self.out = self.recv = None
        if self.rank == dst:
            if self.equal:
                self.out = torch.empty(self.m * len(self.sizes), dtype=dtype, device=device)
                self.recv = list(self.out.split(self.m))
            else:
                self.slots = torch.empty(self.m * len(self.sizes), dtype=dtype, device=device)
                self.recv = list(self.slots.split(self.m))
        self.work = None

    def start(self, t, async_op: bool = False):
        """Gather this rank's counts `t` (sizes[rank] elements) to dst."""
        import torch.distributed as dist

        self.wait()
        n = self.sizes[self.rank]
        if t.numel() < n:
            raise ValueError(f"rank {self.rank}: {t.numel()} counts for a shard of {n}")
        if self.equal:
            src = t[:n] if t.numel() != n else t
        else:
            self.pad[:n].copy_(t[:n])
            src = self.pad
        self.work = dist.gather(src, self.recv if self.rank == self.dst else None, dst=self.dst, group=self.group,
                                async_op=async_op)
        return self.work

    def wait(self) -> None:
        """The pending gather done (on GPUs: the caller's stream waits for it; the host does not block)."""
        if self.work is not None:
            self.work.wait()
            self.work = None

    def result(self):
        """dst: every rank's counts in rank order (a [sum(sizes)] tensor); None elsewhere."""
        import torch

        self.wait()
        if self.rank != self.dst:
            return None
        if self.equal:
            return self.out
        return torch.cat([r[:n] for r, n in zip(self.recv, self.sizes)])


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
