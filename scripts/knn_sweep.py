"""K3 k-NN probe over several context settings in one process: for each
config (NAVGPU_KNN_* env overrides, read at context creation) the isolated
query and build times (HIP events), the slow-path count and, with a stamps
build (--lib .../libnavgpu_stamps.so), the k_knn phase shares.
usage: knn_sweep.py [--lib L] [--reps N] "SX=4,LAMBDA=22" "SX=1" ..."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
import torch  # noqa: E402

import navslam.gpu as G  # noqa: E402
from navslam import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--k", type=int, default=8)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("configs", nargs="*", default=[""])
a = ap.parse_args()
if a.lib:
    G.load_library(a.lib)
dev = torch.device("cuda", 0)
s, t = synth.uniform_pair(512, 2048)
N = s.shape[0] * s.shape[1]
src = torch.from_numpy(s).to(dev)
tgt = torch.from_numpy(t).to(dev)
idx = torch.empty((N, a.k), dtype=torch.int32, device=dev)
dst = torch.empty((N, a.k), dtype=torch.float64, device=dev)
names = ["-", "stage", "queries", "scan", "exact", "n_qwaves", "n_tiles", "barrier", "qsetup", "drain_steps", "drain"]
for cfg in a.configs:
    env = dict(kv.split("=") for kv in cfg.split(",") if kv)
    saved = {}
    for k_, v in env.items():
        saved[k_] = os.environ.get("NAVGPU_KNN_" + k_)
        os.environ["NAVGPU_KNN_" + k_] = v
    os.environ["NAVGPU_KNN_STATS"] = "1"
    g = G.NavGpu(0, torch.cuda.current_stream(dev).cuda_stream)
    g.knn_dev(tgt, N, src, N, a.k, idx, dst)
    torch.cuda.synchronize()
    slow, unstaged = g.knn_fallbacks(), g.knn_overflows()
    g.timing(True)
    for _ in range(a.reps):
        g.knn_dev(tgt, N, src, N, a.k, idx, dst)
    torch.cuda.synchronize()
    q_ms, qn = g.timing_read("knn_query")
    b_ms, bn = g.timing_read("knn_build")
    st = (ctypes.c_ulonglong * 16)()
    stamps = None
    if g.L.navgpu_debug_stamps(st) == 0:
        g.knn_dev(tgt, N, src, N, a.k, idx, dst)
        torch.cuda.synchronize()
        g.L.navgpu_debug_stamps(st)
        stamps = {names[i]: int(st[i]) for i in range(1, 11)}
    print(json.dumps({"cfg": cfg, "lib": os.path.basename(a.lib or "libnavgpu.so"),
                      "query_us": round(1000 * q_ms / qn, 2), "build_us": round(1000 * b_ms / bn, 2),
                      "slow": slow, "unstaged": unstaged, "stamps": stamps}), flush=True)
    g.close()
    for k_, v in saved.items():
        if v is None:
            os.environ.pop("NAVGPU_KNN_" + k_, None)
        else:
            os.environ["NAVGPU_KNN_" + k_] = v
