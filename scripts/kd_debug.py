import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nav-slam_amd"), os.path.join(ROOT, "oracle")]
from navslam.gpu import NavGpu
from pyoracle import Oracle
g = NavGpu(0); o = Oracle()
for n in (70000, 20000, 12000):
    rng = np.random.default_rng(n)
    pts = np.round(rng.uniform(0, 40, (n, 3)))
    t, _ = o.kd_build(pts.copy())
    a = g.kd_build(pts, 0)
    os.environ["NAVGPU_KD_ONE_WG"] = "1"
    b = g.kd_build(pts, 0)
    del os.environ["NAVGPU_KD_ONE_WG"]
    bad = np.where((a != t).any(1))[0]
    badb = np.where((b != t).any(1))[0]
    print(n, "level-par mismatches", len(bad), bad[:20], "one-wg mismatches", len(badb), flush=True)
    if len(bad):
        print(a[bad[:5]], t[bad[:5]])
