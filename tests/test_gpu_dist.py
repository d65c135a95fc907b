"""The K4 exchange through the real RCCL path on the GPU: a world-size-1
`nccl` process group (RCCL on ROCm) on cuda:0, so shard.gather_matches takes
its `all_gather_into_tensor` branch on device buffers. The per-pair match
sets come from the batch kernel (navgpu_rows_match_batch_dev) written
straight into the packed idx + dist buffer (12 B per cell), and
the gathered result is checked against the single-pair host API."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_k4_batch_gather_over_rccl_world1():
    import torch
    import torch.distributed as dist
    from navslam import shard, synth
    from navslam.gpu import NavGpu
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    g = NavGpu(0)
    try:
        assert dist.get_backend() == "nccl"
        R, Cc, pairs = 16, 512, 3
        pmax = pairs + 1          # a padded slot, as the ragged tail of a shard
        ps = [synth.l9_pair(R, Cc, seed=40 + p, integer_mm=(p % 2 == 1)) for p in range(pairs)]
        src = torch.from_numpy(np.stack([p[0] for p in ps])).to(dev)
        tgt = torch.from_numpy(np.stack([p[1] for p in ps])).to(dev)
        packed = torch.empty(pmax * R * Cc * 12, dtype=torch.uint8, device=dev)
        idx, dst = shard.match_views(packed, pmax, R, Cc)
        idx.fill_(-1)
        dst.fill_(float("inf"))
        sm = torch.empty((pmax, R, Cc), dtype=torch.int32, device=dev)
        tm = torch.empty_like(sm)
        torch.cuda.synchronize()
        g.rows_match_batch_dev(src, tgt, pairs, R, Cc, sm, tm, idx, dst)
        g.sync()
        out = shard.gather_matches(packed)
        torch.cuda.synchronize()
        assert out.device == dev and out.numel() == packed.numel()
        gi, gd = shard.unpack_gathered(out, 1, pmax, R, Cc)
        for p in range(pairs):
            _, _, ni, nd = g.rows_match(ps[p][0], ps[p][1])
            np.testing.assert_array_equal(gi[p].cpu().numpy(), ni)
            np.testing.assert_array_equal(gd[p].cpu().numpy(), nd)
        assert (gi[pairs] == -1).all() and torch.isinf(gd[pairs]).all()
        assert shard.max_over_ranks(1.5, dev) == 1.5
        assert shard.sum_over_ranks(pairs, dev) == pairs
    finally:
        g.close()
        dist.destroy_process_group()
