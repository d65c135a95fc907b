"""Per-row build phases (NAVGPU_STAMPS builds): times navgpu_kd_build_rows_dev
on K2-shaped L9 frames and prints the s_memtime phase sums of
row_stage_and_build / block_build_kdtree (slots 8-12), per row."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
import torch  # noqa: E402

from navslam import synth  # noqa: E402
import navslam.gpu as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--rows", type=int, default=128)
ap.add_argument("--cols", type=int, default=2048)
ap.add_argument("--integer", action="store_true")
a = ap.parse_args()
if a.lib:
    G.load_library(a.lib)
dev = torch.device("cuda", 0)
g = G.NavGpu(0, torch.cuda.current_stream(dev).cuda_stream)
R, Cc = a.rows, a.cols
s, t = synth.l9_pair(R, Cc, seed=5, integer_mm=a.integer)
tgt = torch.from_numpy(t).to(dev)
tp = torch.empty((R, Cc, 3), dtype=torch.float64, device=dev)
tc = torch.empty((R, Cc), dtype=torch.int32, device=dev)
tn = torch.empty((R,), dtype=torch.int32, device=dev)
for _ in range(2):
    g.kd_build_rows_dev(tgt, tgt, R, Cc, tp, tc, tn)
torch.cuda.synchronize()
st = (ctypes.c_ulonglong * 16)()
have = g.L.navgpu_debug_stamps(st) == 0
g.timing(True)
g.kd_build_rows_dev(tgt, tgt, R, Cc, tp, tc, tn)
torch.cuda.synchronize()
ms, n = g.timing_read("rows_build")
out = {"lib": os.path.basename(a.lib or "libnavgpu.so"), "build_us": 1000 * ms / max(n, 1),
       "mean_features": float(tn.float().mean()), "max_features": int(tn.max())}
if have:
    g.L.navgpu_debug_stamps(st)
    nb = max(int(st[12]), 1)
    # s_memtime ticks per row (shader clock); shares of the row's build
    ph = {k: int(st[i]) / nb for i, k in ((8, "stage"), (9, "root"), (10, "wave_levels"),
                                          (11, "lane_subtrees"))}
    tot = sum(ph.values()) or 1
    out.update({k + "_ticks_per_row": round(v) for k, v in ph.items()})
    out.update({k + "_share": round(v / tot, 3) for k, v in ph.items()})
    out["rows"] = nb
print(json.dumps(out))
