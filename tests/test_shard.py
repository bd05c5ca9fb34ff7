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
