"""k_rows_screen phase stamps (a -DNAVGPU_STAMPS build, --lib): per-wave
s_memtime sums of the target compaction, the chunk boxes, the query
compaction and the query loop, chunk scans per query wave."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
import torch  # noqa: E402

from navslam import synth  # noqa: E402
import navslam.gpu as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
ap.add_argument("--pairs", type=int, default=8)
a = ap.parse_args()
G.load_library(a.lib)
dev = torch.device("cuda", 0)
g = G.NavGpu(0)
R, Cc, P = 128, 2048, a.pairs
pairs = [synth.l9_pair(R, Cc, seed=p + 5) for p in range(P)]
src = torch.stack([torch.from_numpy(x) for x, _ in pairs]).to(dev)
tgt = torch.stack([torch.from_numpy(y) for _, y in pairs]).to(dev)
i32 = lambda: torch.empty((P, R, Cc), dtype=torch.int32, device=dev)  # noqa: E731
sm, tm, idx = i32(), i32(), i32()
dst = torch.empty((P, R, Cc), dtype=torch.float64, device=dev)
for env in ({}, {"NAVGPU_SCREEN_S": "4"}):
    for k in ("NAVGPU_SCREEN_S",):
        os.environ.pop(k, None)
    os.environ.update(env)
    g.rows_match_batch_dev(src, tgt, P, R, Cc, sm, tm, idx, dst)
    torch.cuda.synchronize()
    st = (ctypes.c_ulonglong * 16)()
    g.L.navgpu_debug_stamps(st)
    g.rows_match_batch_dev(src, tgt, P, R, Cc, sm, tm, idx, dst)
    torch.cuda.synchronize()
    g.L.navgpu_debug_stamps(st)
    v = list(st)
    nw = v[14]
    print(env, f"waves(query iters) {nw}, chunk scans/wave {v[13] / max(nw, 1):.2f}; "
          f"per wave-slot cycles: tgt compact {v[0]}, boxes {v[1]}, q compact {v[2]}, "
          f"query loop {v[3]}  (sums over all waves); query loop per iter {v[3] / max(nw, 1):.0f}",
          flush=True)
