"""Multi-rank path on CPU (gloo, world_size 2): contiguous pattern shards searched
independently and gathered in rank order reproduce the single-process result."""
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT
import edsgen


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, base, buf, offs, q):
    import importlib
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc

    shard = importlib.import_module("eds-bwt_amd.shard")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, o, first = shard.shard_patterns(buf, offs, world, rank)
    counts, occ, _ = orc.Engine(base).search(b, o, first_pattern_id=first)  # stands in for the GPU search on CPU
    # the exchange step bench.py runs over RCCL: sizes all-gathered, counts and 20-B records
    # gathered to rank 0 as padded tensors
    sizes = shard.exchange_sizes(counts.size, occ.size, "cpu")
    npats = [int(x) for x in sizes[:, 0]]
    noccs = [int(x) for x in sizes[:, 1]]
    assert sum(npats) == offs.size - 1
    allc = shard.gather_counts(torch.from_numpy(counts.astype(np.int32)), npats)
    rec = torch.from_numpy(occ.view(np.uint32).reshape(-1).view(np.int32).copy())
    allocc = shard.gather_records(rec, noccs)
    if rank == 0:
        q.put((allc.numpy(), shard.records_to_numpy(allocc)))
    else:
        assert allc is None and allocc is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_single(oracle, tmp_path, world):
    rng = random.Random(world)
    segs = edsgen.random_eds(rng, 300, p_empty=0.2)
    (tmp_path / "s.eds").write_text(edsgen.eds_text(segs))
    base = str(tmp_path / "s")
    oracle.transform(str(tmp_path / "s.eds"), base)
    pats = [edsgen.planted(rng, segs, rng.randint(3, 15)) or "ACGT" for _ in range(101)]
    buf = np.frombuffer("".join(pats).encode(), np.uint8).copy()
    offs = np.concatenate(([0], np.cumsum([len(p) for p in pats]))).astype(np.uint64)
    ref_counts, ref_occ, _ = oracle.Engine(base).search(buf, offs)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, base, buf, offs, q)) for r in range(world)]
    for p in procs:
        p.start()
    counts, occ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(counts.astype(np.uint32), ref_counts)
    assert np.array_equal(occ, ref_occ)


def _exchange_worker(rank, world, port, sizes, q):
    import importlib
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    shard = importlib.import_module("eds-bwt_amd.shard")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo = sum(sizes[:rank])
    sx = shard.SizesExchange("cpu")
    cg = shard.CountsGather(sizes, "cpu")
    # the per-step exchange of bench.py, repeated over alternating buffers (the timed steps reuse
    # them): each step's counts are lo + i + 1000 * step, only the last gather is kept
    bufs = [torch.zeros(sizes[rank], dtype=torch.int32) for _ in range(2)]
    for step in range(5):
        b = bufs[step % 2]
        b.copy_(torch.arange(lo, lo + sizes[rank], dtype=torch.int32) + 1000 * step)
        sx.start(sizes[rank], 7 * (rank + 1) + step, async_op=True)
        cg.start(b, async_op=True)
    out = cg.result()
    sz = sx.result()
    if rank == 0:
        q.put((out.numpy().copy(), sz.numpy().copy()))
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,sizes", [(2, [5, 5]), (3, [4, 4, 4]), (3, [3, 4, 0]), (2, [0, 6])])
def test_counts_gather_and_sizes_exchange(world, sizes):
    """bench.py's per-step exchange (shard.CountsGather / SizesExchange, set up once per batch
    shape): after repeated asynchronous steps rank 0 holds every rank's last counts in rank order
    (equal shards: received into slices of one tensor; unequal: padded slots, compacted) and the
    last (patterns, records) of every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    counts, sz = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(counts, np.arange(sum(sizes), dtype=np.int32) + 4000)
    assert sz.tolist() == [[sizes[r], 7 * (r + 1) + 4] for r in range(world)]
