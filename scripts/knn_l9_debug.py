"""Mismatches of the global k-NN on an L9-shaped pair against the oracle's
grid and brute-force k-NN (debug helper for test_knn_global_on_l9_scan)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nav-slam_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
from pyoracle import Oracle  # noqa: E402

from navslam.gpu import NavGpu  # noqa: E402
from navslam.synth import l9_pair  # noqa: E402

im = len(sys.argv) > 1 and sys.argv[1] == "int"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
src, tgt = l9_pair(128, 2048, seed=21, integer_mm=im)
g = NavGpu(0)
orc = Oracle()
gi, gd = g.knn(tgt, src, k)
ri, rd = orc.knn_grid(tgt, src, k)
bad = np.nonzero((gi != ri).any(1) | (gd != rd).any(1))[0]
print("mismatched queries", len(bad))
q = src.reshape(-1, 3)
t = tgt.reshape(-1, 3)
for b in bad[:8]:
    bi, bd = orc.knn_brute(tgt, q[b:b + 1], k)
    print("q", b, q[b].tolist())
    print("  gpu  ", gi[b].tolist(), gd[b].tolist())
    print("  grid ", ri[b].tolist(), rd[b].tolist())
    print("  brute", bi[0].tolist(), bd[0].tolist())
    for j in sorted(set(gi[b].tolist()) ^ set(ri[b].tolist())):
        if j >= 0:
            print("   pt", j, t[j].tolist(), float(np.sqrt(((t[j] - q[b]) ** 2).sum())))
