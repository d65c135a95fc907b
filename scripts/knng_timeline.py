"""k_knng per-chunk timeline (stamps variant build, -DNAVGPU_STAMPS): wave
durations, phase cycles, and how many waves each SIMD held over the kernel.
  python3 scripts/knng_timeline.py --lib nav-slam_amd/lib/variants/libnavgpu_stamps.so"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
ap.add_argument("--k", type=int, default=8)
a = ap.parse_args()
import navslam.gpu as _g  # noqa: E402
_g.load_library(a.lib)
import torch  # noqa: E402
from navslam import synth  # noqa: E402
from navslam.gpu import NavGpu  # noqa: E402

dev = torch.device("cuda", 0)
g = NavGpu(0, torch.cuda.current_stream(dev).cuda_stream)
s, t = synth.uniform_pair(512, 2048)
N = s.shape[0] * s.shape[1]
src = torch.from_numpy(s).to(dev)
tgt = torch.from_numpy(t).to(dev)
idx = torch.empty((N, a.k), dtype=torch.int32, device=dev)
dst = torch.empty((N, a.k), dtype=torch.float64, device=dev)
for _ in range(3):
    g.knn_dev(tgt, N, src, N, a.k, idx, dst)
torch.cuda.synchronize()
L = g.L
L.navgpu_debug_knng_timeline.restype = ctypes.c_int
L.navgpu_debug_knng_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
nch = (N + 63) // 64
buf = np.zeros((nch, 8), np.uint64)
assert L.navgpu_debug_knng_timeline(buf.ctypes.data, nch) == nch
t0 = buf[:, 0].astype(np.int64)
t1 = buf[:, 1].astype(np.int64)
hw = buf[:, 2].astype(np.int64)
xcc = buf[:, 3].astype(np.int64) & 0xf
base = t0.min()
t0 -= base
t1 -= base
dur = (t1 - t0) * 10.0 / 1000  # us (100 MHz)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
slot = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
nsl = len(np.unique(slot))
span = (t1.max() - t0.min()) * 10.0 / 1000
busy = (t1 - t0).sum() * 10.0 / 1000
out = {
    "chunks": int(nch), "span_us": span, "wave_us_mean": float(dur.mean()),
    "wave_us_p10_p50_p90": [float(np.percentile(dur, p)) for p in (10, 50, 90)],
    "simds_seen": int(nsl), "mean_waves_per_simd": busy / (span * nsl),
    "rounds_mean": float(buf[:, 7].astype(np.float64).mean()),
    "cycles_stage_scan_exact_mean": [float(buf[:, i].astype(np.float64).mean()) for i in (4, 5, 6)],
}
# per XCD spans
out["xcd_end_us"] = [float(t1[xcc == x].max() * 10.0 / 1000) for x in range(8)]
out["xcd_start_us"] = [float(t0[xcc == x].min() * 10.0 / 1000) for x in range(8)]
# concurrency over time (all SIMDs): sample 200 points
ts = np.linspace(0, t1.max(), 200)
conc = [int(((t0 <= x) & (t1 > x)).sum()) for x in ts]
out["concurrent_waves_by_time"] = conc[::10]
print(json.dumps(out))
