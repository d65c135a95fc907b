"""navgpu_debug_nth_element (one wave / the block pass) against plain Lomuto (tests/test_lomuto_models.py)
on random, sorted, scan-like and duplicate-heavy windows; prints the first
failures and saves them under gpurun_out/nth_debug/."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "nav-slam_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import navslam.gpu as G  # noqa: E402
from test_lomuto_models import lomuto_nth, _keys  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1].endswith(".so"):
    G.load_library(sys.argv[1])
dev = torch.device("cuda", 0)
g = G.NavGpu(0, torch.cuda.current_stream(dev).cuda_stream)
out = os.path.join(ROOT, "gpurun_out", "nth_debug")
os.makedirs(out, exist_ok=True)
rng = np.random.default_rng(7)
fails = 0
cases = 0
for kind in ("random", "sorted", "reversed", "duplicates", "scanlike"):
    for trial in range(40):
        n = int(rng.integers(65, 1600)) if trial % 4 else int(rng.integers(65, 200))
        key = (list(np.cumsum(rng.normal(-0.3, 1.0, n))) if kind == "scanlike"
               else _keys(rng, kind, n))
        P0 = list(rng.permutation(n))
        first = int(rng.integers(0, max(1, n // 4)))
        last = int(rng.integers(first + 1, n))
        nth = int(rng.integers(first, last + 1))
        ref = P0.copy()
        lomuto_nth(key, ref, first, last, nth)
        for block in (0, 1):
            kd = torch.tensor(key, dtype=torch.float64, device=dev)
            pd = torch.tensor(P0, dtype=torch.int32, device=dev)
            g.debug_nth_element(kd, pd, first, last, nth, block=bool(block))
            torch.cuda.synchronize()
            got = pd.cpu().tolist()
            cases += 1
            if got != ref:
                fails += 1
                bad = [i for i in range(n) if got[i] != ref[i]]
                if fails <= 6:
                    print(f"FAIL {kind} n={n} first={first} last={last} nth={nth} block={block} "
                          f"bad={len(bad)} at {bad[:12]} dup={len(got) - len(set(got))}", flush=True)
                    np.savez(os.path.join(out, f"fail{fails}.npz"), key=np.array(key), P0=np.array(P0),
                             first=first, last=last, nth=nth, block=block, got=np.array(got),
                             ref=np.array(ref))
print(f"{'OK' if not fails else 'BAD'} {cases - fails}/{cases} cases")
sys.exit(1 if fails else 0)
