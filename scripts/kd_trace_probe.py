"""Per-level quickselect iteration trace of the large buildKDTree
(NAVGPU_KD_TRACE=1), two builds of the same points in a row."""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "nav-slam_amd")]
from navslam.gpu import NavGpu  # noqa: E402

os.environ["NAVGPU_KD_TRACE"] = "1"
g = NavGpu(0)
pts = np.random.default_rng(1).uniform(0, 1000, (1 << 20, 3))
a = g.kd_build(pts, 0)
print("---- second build", flush=True)
b = g.kd_build(pts, 0)
print("same result:", bool((a == b).all()), flush=True)
