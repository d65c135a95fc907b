"""K2 per-row mode timing split: fused k_rows_match vs k_rows_build +
k_rows_query (torch events on the library's stream)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
import torch  # noqa: E402
from navslam import synth  # noqa: E402
import navslam.gpu as ng  # noqa: E402
from navslam.gpu import NavGpu  # noqa: E402

if len(sys.argv) > 1:  # --lib path: an experimental build
    ng.load_library(sys.argv[1])

R, C = 128, 2048
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
g = NavGpu(0, st.cuda_stream)
s_h, t_h = synth.l9_pair(R, C, seed=5)
src = torch.from_numpy(s_h).to(dev)
tgt = torch.from_numpy(t_h).to(dev)
i32 = lambda: torch.empty((R, C), dtype=torch.int32, device=dev)  # noqa: E731
sm, tm, idx = i32(), i32(), i32()
dst = torch.empty((R, C), dtype=torch.float64, device=dev)
tp = torch.empty((R, C, 3), dtype=torch.float64, device=dev)
tc, pos = i32(), i32()
tn = torch.empty(R, dtype=torch.int32, device=dev)


def timeit(fn, reps=20):
    # the library runs on its own stream when handed torch's default (null)
    # stream, so time with device-wide synchronisation
    import time
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / reps


out = {
    "rows_match_us": timeit(lambda: g.rows_match_dev(src, tgt, R, C, sm, tm, idx, dst)),
    "rows_build_us": timeit(lambda: g.kd_build_rows_dev(tgt, tgt, R, C, tp, tc, tn, tm)),
    "rows_query_us": timeit(lambda: g.kd_query_rows_dev(tp, tn, src, src, R, C, pos, dst, sm)),
    "tree_n_mean": float(tn.float().mean().item()),
    "queries_mean": float(sm.float().sum(1).mean().item()),
}
out["lib"] = os.path.basename(sys.argv[1]) if len(sys.argv) > 1 else "libnavgpu.so"
import ctypes  # noqa: E402
st = (ctypes.c_ulonglong * 16)()
if g.L.navgpu_debug_stamps(st) == 0:  # NAVGPU_STAMPS builds: one clean build call
    g.kd_build_rows_dev(tgt, tgt, R, C, tp, tc, tn, tm)
    torch.cuda.synchronize()
    g.L.navgpu_debug_stamps(st)
    nb = max(int(st[12]), 1)
    out["stamps_cycles_per_row"] = {"stage+curv+compact": int(st[8]) // nb,
                                    "root(block)": int(st[9]) // nb,
                                    "wave levels": int(st[10]) // nb,
                                    "lane tail": int(st[11]) // nb, "rows": nb}
print(json.dumps(out))
