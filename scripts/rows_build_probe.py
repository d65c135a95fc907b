"""k_rows_build on K5 frames: kernel time (HIP events on the context's
stream) and, for a -DNAVGPU_STAMPS build (--lib), the per-workgroup phase
split of row_stage_and_build / block_build_kdtree (stamp slots 8-11:
stage+compact, block-wide levels, wave levels, lane subtrees)."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from navslam import synth  # noqa: E402
import navslam.gpu as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--tag", default="")
a = ap.parse_args()
if a.lib:
    G.load_library(a.lib)
dev = torch.device("cuda", 0)
g = G.NavGpu(0)
g.L.navgpu_debug_stamps.argtypes = [ctypes.c_void_p]
R, Cc = 128, 2048
fr = torch.from_numpy(synth.l9_stream(R, Cc, frames=a.frames)).to(dev)
tree = torch.empty((R, Cc, 3), dtype=torch.float64, device=dev)
tcol = torch.empty((R, Cc), dtype=torch.int32, device=dev)
tn = torch.empty(R, dtype=torch.int32, device=dev)
st = (ctypes.c_ulonglong * 16)()
out = {"lib": os.path.basename(a.lib or "default"), "tag": a.tag}
for f in range(a.frames):
    g.kd_build_rows_dev(fr[f], fr[f], R, Cc, tree, tcol, tn)
g.sync()
stamps = g.L.navgpu_debug_stamps(st) == 0
g.L.navgpu_timing_enable(g.h, 1)
g.L.navgpu_timing_read(g.h, b"rows_build", 1)
for i in range(a.reps):
    f = i % a.frames
    g.kd_build_rows_dev(fr[f], fr[f], R, Cc, tree, tcol, tn)
g.sync()
ms = g.L.navgpu_timing_read(g.h, b"rows_build", 1)
out["us_per_build"] = round(1e3 * ms / a.reps, 2)
out["features_per_row"] = float(tn.float().mean().item())
if stamps:
    g.L.navgpu_debug_stamps(st)
    wg = R * a.reps
    names = {8: "stage", 9: "block_levels", 10: "wave_levels", 11: "lane_subtrees"}
    out["cycles_per_wg"] = {names[k]: round(st[k] / wg) for k in names}
    out["block_per_wg"] = {"passes": st[13] / wg, "chunks": st[14] / wg, "xwave_rounds": st[15] / wg}
print(json.dumps(out))
