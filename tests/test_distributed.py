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
        pmax = -(-pairs // world)
        # the rank's match sets packed as bench.py's K4 does: idx then dist,
        # 12 B per cell, pmax slots (a ragged tail leaves the last slot unused)
        packed = torch.zeros(pmax * R * Cc * 12, dtype=torch.uint8)
        idx, dst = shard.match_views(packed, pmax, R, Cc)
        idx.fill_(-1)
        for i, p in enumerate(range(lo, hi)):
            src, tgt = synth.l9_pair(R, Cc, seed=100 + p, integer_mm=True)
            _, _, ni, nd = orc.rows_match(src, tgt)
            idx[i] = torch.from_numpy(ni)
            dst[i] = torch.from_numpy(nd)
        out = shard.gather_matches(packed)
        gi, gd = shard.unpack_gathered(out, world, pmax, R, Cc)
        slowest = shard.max_over_ranks(0.25 * (rank + 1), torch.device("cpu"))
        total = shard.sum_over_ranks(hi - lo, torch.device("cpu"))
        if rank == 0:
            q.put((gi.numpy(), gd.numpy(), slowest, total))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pairs", [4, 5])
def test_k4_shard_and_gather_gloo_world2(orc, pairs):
    """K4 plumbing at world 2 (gloo): contiguous shards, one all-gather of the
    packed idx + dist match sets, a ragged tail (5 pairs over 2 ranks) padded;
    the gathered sets equal a single-process run pair by pair."""
    world, R, Cc = 2, 6, 64
    q = mp.get_context("spawn").SimpleQueue()
    mp.spawn(_worker, args=(world, _free_port(), pairs, R, Cc, q), nprocs=world, join=True)
    gi, gd, slowest, total = q.get()
    assert slowest == 0.5 and total == pairs
    pmax = -(-pairs // world)
    assert gi.shape == (world * pmax, R, Cc)
    for p in range(pairs):
        r = 0 if p < pmax else 1
        slot = r * pmax + (p - shard.shard_pairs(pairs, world, r)[0])
        _, _, ni, nd = orc.rows_match(*synth.l9_pair(R, Cc, seed=100 + p, integer_mm=True))
        np.testing.assert_array_equal(gi[slot], ni)
        np.testing.assert_array_equal(gd[slot], nd)
    used = {r * pmax + i for r in range(world)
            for i in range(np.subtract(*shard.shard_pairs(pairs, world, r)[::-1]))}
    for slot in set(range(world * pmax)) - used:   # padding of the ragged tail
        assert (gi[slot] == -1).all()


def _bench_cmd(*extra):
    import sys
    return [sys.executable, os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"),
            "--dry-run", "--workload", "k4", "--pairs", "5"] + list(extra)


def test_bench_gpus_launches_that_many_ranks():
    """`bench.py --gpus 2` without a launcher starts 2 ranks itself (a
    torch.distributed.run child), and both report (gloo, no GPU)."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run(_bench_cmd("--gpus", "2"), env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    out = lines[0]
    assert out["n_gpus"] == 2 and out["gpus_requested"] == 2
    assert sorted(x[0] for x in out["ranks_reported"]) == [0, 1]
    assert [x[1:] for x in sorted(out["ranks_reported"])] == [[0, 3], [3, 5]]
    assert out["pairs"] == 5


def test_bench_world_size_mismatch_is_an_error():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run(_bench_cmd("--gpus", "2"), env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
