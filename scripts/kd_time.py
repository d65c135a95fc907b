"""Times buildKDTree (navgpu_kd_build_dev, device-resident) at 1M points:
the level-parallel build and the single-workgroup one (NAVGPU_KD_ONE_WG);
the reference's own buildKDTree (utils/kdtree.c:65-82) time comes from
oracle/_ref when present on the host, else the oracle restatement."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nav-slam_amd"), os.path.join(ROOT, "oracle")]
import torch  # noqa: E402

from navslam.gpu import NavGpu  # noqa: E402
from pyoracle import Oracle  # noqa: E402

dev = torch.device("cuda", 0)
g = NavGpu(0)
g.timing(True)
out = {}
for n in (1 << 20, 1 << 17):
    rng = np.random.default_rng(1)
    h = rng.uniform(0, 1000, (n, 3))
    src = torch.from_numpy(h).to(dev)
    buf = torch.empty_like(src)
    for mode in ("level_parallel", "one_workgroup"):
        if mode == "one_workgroup":
            os.environ["NAVGPU_KD_ONE_WG"] = "1"
        reps = 5
        for r in range(reps + 1):
            buf.copy_(src)
            torch.cuda.synchronize()  # the library runs on its own stream
            if r == 1:
                g.timing_read("kd_build")
            g.kd_build_dev(buf, n, 0)
            g.sync()
        torch.cuda.synchronize()
        ms, k = g.timing_read("kd_build")
        out[f"n{n}_{mode}_ms"] = round(ms / k, 3)
        os.environ.pop("NAVGPU_KD_ONE_WG", None)
    o = Oracle()
    t0 = time.perf_counter()
    o.kd_build(h.copy())
    out[f"n{n}_cpu_oracle_ms"] = round(1e3 * (time.perf_counter() - t0), 1)
print(json.dumps(out))
