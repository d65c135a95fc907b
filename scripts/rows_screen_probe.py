"""Time rows_match (screened per-row path) over screen launch knobs
(NAVGPU_SCREEN_S / NAVGPU_SCREEN_NT are read per call) on the K2 pair and a
K4-style batch; prints one line per configuration."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nav-slam_amd"), ROOT]
import torch  # noqa: E402

from navslam import synth  # noqa: E402
import navslam.gpu as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--default-only", action="store_true")
args = ap.parse_args()
if args.lib:
    G.load_library(args.lib)
NavGpu = G.NavGpu
dev = torch.device("cuda", 0)
g = NavGpu(0)
g.timing(True)
R, Cc = 128, 2048


def run(P, reps, label):
    pairs = [synth.l9_pair(R, Cc, seed=p + 5) for p in range(min(P, 8))]
    src = torch.stack([torch.from_numpy(pairs[p % len(pairs)][0]) for p in range(P)]).to(dev)
    tgt = torch.stack([torch.from_numpy(pairs[p % len(pairs)][1]) for p in range(P)]).to(dev)
    i32 = lambda: torch.empty((P, R, Cc), dtype=torch.int32, device=dev)  # noqa: E731
    sm, tm, idx = i32(), i32(), i32()
    dst = torch.empty((P, R, Cc), dtype=torch.float64, device=dev)
    confs = [(None, None)] if args.default_only else [
        (None, None), ("1", None), ("2", None), ("4", None), ("8", None), ("16", None),
        ("2", "512"), ("4", "512"), ("1", "512")]
    for s_, nt in confs:
        for k, v in (("NAVGPU_SCREEN_S", s_), ("NAVGPU_SCREEN_NT", nt)):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        g.rows_match_batch_dev(src, tgt, P, R, Cc, sm, tm, idx, dst)
        torch.cuda.synchronize()
        g.timing_read("rows_match")
        t0 = time.perf_counter()
        for _ in range(reps):
            g.rows_match_batch_dev(src, tgt, P, R, Cc, sm, tm, idx, dst)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps * 1e3
        ms, n = g.timing_read("rows_match")
        print(f"{label} P={P} S={s_} NT={nt}: kernel {ms / n * 1e3:.1f} us/call, wall {wall:.3f} ms, "
              f"tie rows {g.rows_tie_rows()}", flush=True)


run(1, 30, "K2")
run(32, 5, "K4-32")
