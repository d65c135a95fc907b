"""K2 phases (NAVGPU_STAMPS builds): rows_match on a K2-shaped L9 pair, then
the f32 screen's counters (waves, waves with an f64 fallback, fallback
lanes, chunks scanned past the first two: slots 0-3) and the tie pass's
s_memtime sums per building row: stage + build (slot 4; 8-12 split it) and
the source staging + walk (slot 5), the queries walked (6), the rows that
built (7)."""
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
ap.add_argument("--integer", action="store_true")
a = ap.parse_args()
if a.lib:
    G.load_library(a.lib)
g = G.NavGpu(0)
s, t = synth.l9_pair(128, 2048, seed=5, integer_mm=a.integer)
for _ in range(2):
    g.rows_match(s, t)
st = (ctypes.c_ulonglong * 16)()
g.L.navgpu_debug_stamps(st)  # reset
g.timing(True)
g.rows_match(s, t)
torch.cuda.synchronize()
ms, n = g.timing_read("rows_match")
have = g.L.navgpu_debug_stamps(st) == 0
out = {"lib": os.path.basename(a.lib or "libnavgpu.so"), "rows_match_us": 1000 * ms / max(n, 1)}
if have:
    out["slots"] = [int(x) for x in st]
    out.update({"screen_waves": int(st[0]), "fallback_waves": int(st[1]),
                "fallback_lanes": int(st[2]), "extra_chunks_per_wave": round(st[3] / max(st[0], 1), 2)})
    nb = max(int(st[7]), 1)
    out.update({"rows_built": int(st[7]), "walked_per_row": round(st[6] / nb, 1),
                "build_ticks_per_row": round(st[4] / nb), "walk_ticks_per_row": round(st[5] / nb),
                "root_ticks_per_row": round(st[9] / nb), "wave_levels_ticks_per_row": round(st[10] / nb),
                "lane_ticks_per_row": round(st[11] / nb)})
print(json.dumps(out))
