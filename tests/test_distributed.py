"""N > 1 plumbing on the CPU: gloo, world_size 2, the same helpers bench.py
uses on the GPU box (navslam.shard). The per-pair compute is the oracle's
per-row matcher standing in for the GPU kernel (test infrastructure), so the
sharded + gathered result can be checked against a single-process run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from navslam import shard, synth


def test_shard_pairs_cover_and_are_contiguous():
    for total in (0, 1, 7, 8, 256, 257):
        for world in (1, 2, 3, 8):
            spans = [shard.pair_seeds(r) for r in range(world)]
            assert len(set(spans)) == world  # distinct seeds per rank
            got = [shard.shard_pairs(total, world, r) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == total
            for (a, b), (c, d) in zip(got, got[1:]):
                assert b == c and a <= b
            sizes = [b - a for a, b in got]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_pairs(4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, pairs, R, Cc, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pyoracle import Oracle
        orc = Oracle()
        lo, hi = shard.shard_pairs(pairs, world, rank)
        local = np.zeros((hi - lo, R, Cc), np.int32)
        for i, p in enumerate(range(lo, hi)):
            src, tgt = synth.l9_pair(R, Cc, seed=100 + p, integer_mm=True)
            local[i] = orc.rows_match(src, tgt)[2]
        out = shard.gather_matches(torch.from_numpy(local))
        slowest = shard.max_over_ranks(0.25 * (rank + 1), torch.device("cpu"))
        total = shard.sum_over_ranks(hi - lo, torch.device("cpu"))
        if rank == 0:
            q.put((out.numpy(), slowest, total))
    finally:
        dist.destroy_process_group()


def test_k4_shard_and_gather_gloo_world2(orc):
    world, pairs, R, Cc = 2, 4, 6, 64
    q = mp.get_context("spawn").SimpleQueue()
    mp.spawn(_worker, args=(world, _free_port(), pairs, R, Cc, q), nprocs=world, join=True)
    gathered, slowest, total = q.get()
    assert slowest == 0.5 and total == pairs
    ref = np.stack([orc.rows_match(*synth.l9_pair(R, Cc, seed=100 + p, integer_mm=True))[2]
                    for p in range(pairs)])
    assert gathered.shape == ref.shape
    assert np.array_equal(gathered, ref)
