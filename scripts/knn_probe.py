"""Times the K3 k-NN pieces at the current NAVGPU_KNN_OCC and reports the
slow-path count (NAVGPU_KNN_STATS=1)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
import torch  # noqa: E402

from navslam import synth  # noqa: E402
from navslam.gpu import NavGpu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--occ", default=os.environ.get("NAVGPU_KNN_OCC", "3"))
ap.add_argument("--k", type=int, default=8)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--lib", default=None, help="alternative libnavgpu.so (variant build)")
a = ap.parse_args()
if a.lib:
    import navslam.gpu as _g
    _g.load_library(a.lib)
dev = torch.device("cuda", 0)
g = NavGpu(0, torch.cuda.current_stream(dev).cuda_stream)
s, t = synth.uniform_pair(512, 2048)
N = s.shape[0] * s.shape[1]
src = torch.from_numpy(s).to(dev)
tgt = torch.from_numpy(t).to(dev)
idx = torch.empty((N, a.k), dtype=torch.int32, device=dev)
dst = torch.empty((N, a.k), dtype=torch.float64, device=dev)
g.knn_dev(tgt, N, src, N, a.k, idx, dst)
torch.cuda.synchronize()
slow = g.knn_fallbacks()
ovf = g.knn_overflows() if hasattr(g.L, "navgpu_knn_overflows") else -1
g.timing(True)
for _ in range(a.reps):
    g.knn_dev(tgt, N, src, N, a.k, idx, dst)
torch.cuda.synchronize()
q_ms, qn = g.timing_read("knn_query")
import ctypes  # noqa: E402
st = (ctypes.c_ulonglong * 16)()
stamps = None
if hasattr(g.L, "navgpu_debug_stamps") and g.L.navgpu_debug_stamps(st) == 0:
    # rerun one call with clean stamps
    g.knn_dev(tgt, N, src, N, a.k, idx, dst)
    torch.cuda.synchronize()
    g.L.navgpu_debug_stamps(st)
    names = ["-", "tile_setup+stage", "tile_queries", "q_scan", "q_exact", "n_q_waves", "n_tiles",
             "tile_barrier"]
    stamps = {names[i]: int(st[i]) for i in range(1, 8)}
    stamps["raw"] = [int(st[i]) for i in range(16)]
b_ms, bn = g.timing_read("knn_build")
print(json.dumps({"lib": os.path.basename(a.lib or "libnavgpu.so"), "occ": float(a.occ), "k": a.k, "query_us": 1000 * q_ms / qn,
                  "build_us": 1000 * b_ms / bn, "slow_lanes": slow,
                  "slow_frac": slow / N, "ovf_chunks": ovf, "stamps": stamps}))
