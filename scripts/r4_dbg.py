import sys, os, numpy as np
sys.path.insert(0, "nav-slam_amd")
import navslam.gpu as G
G.load_library("nav-slam_amd/lib/variants/libnavgpu_check.so")
from navslam.gpu import NavGpu
g = NavGpu(0)
rng = np.random.default_rng(1)
tgt, q = rng.uniform(0, 1000, (5000, 3)), rng.uniform(-50, 1050, (3000, 3))
try:
    gi, gd = g.knn(tgt, q, 1)
    print("ok", gi[:3].ravel())
except Exception as e:
    print("ERR", e)
