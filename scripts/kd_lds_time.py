"""buildKDTree in one workgroup's LDS (k_kd_build_lds) at n =
3000-5600, with this library and a variant (--lib) built without the
block-level loop (NAVGPU_KD_LDS_NOLEVELS). Prints ms per build."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nav-slam_amd")]
import torch  # noqa: E402

import navslam.gpu as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
a = ap.parse_args()
if a.lib:
    G.load_library(a.lib)
dev = torch.device("cuda", 0)
g = G.NavGpu(0)
g.timing(True)
out = {"lib": os.path.basename(a.lib or "libnavgpu.so")}
for n in (3000, 4000, 5000, 5600):
    rows = []
    for seed in range(4):
        h = np.random.default_rng(seed).uniform(0, 1000, (n, 3))
        src = torch.from_numpy(h).to(dev)
        buf = torch.empty_like(src)
        for r in range(6):
            buf.copy_(src)
            torch.cuda.synchronize()
            if r == 1:
                g.timing_read("kd_build")
            g.kd_build_dev(buf, n, 0)
            g.sync()
        ms, k = g.timing_read("kd_build")
        rows.append(ms / k)
    out[f"n{n}_us"] = round(1000 * float(np.median(rows)), 1)
print(json.dumps(out))
