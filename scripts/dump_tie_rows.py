"""The K2i target rows (bench --workload k2 --integer-mm, seed 5) as feature
lists for scripts/lomuto_pass_stats.c: int rows, then per row int n and n x 3 f64."""
import sys, struct, numpy as np
sys.path[:0] = ["nav-slam_amd", "oracle"]
from navslam import synth
from pyoracle import Oracle
orc = Oracle()
R, C = 128, 2048
s, t = synth.l9_pair(R, C, seed=5, integer_mm=True)
feat = orc.extract_feature(t)
feat = np.asarray(feat).reshape(R, C)
with open(sys.argv[1], "wb") as f:
    f.write(struct.pack("i", R))
    ns = []
    for r in range(R):
        rows = np.ascontiguousarray(t.reshape(R, C, 3)[r][feat[r] != 0], np.float64)
        ns.append(len(rows))
        f.write(struct.pack("i", len(rows))); f.write(rows.tobytes())
print("n per row: min %d median %d max %d" % (min(ns), int(np.median(ns)), max(ns)))
