"""STREAM-copy ceiling of libnavgpu's k_stream_copy (1 GiB -> 1 GiB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
import torch  # noqa: E402

import navslam.gpu as G  # noqa: E402

if len(sys.argv) > 1:
    G.load_library(sys.argv[1])
g = G.NavGpu(0)
nb = 1 << 30
a = torch.ones(nb, dtype=torch.uint8, device="cuda")
b = torch.empty(nb, dtype=torch.uint8, device="cuda")
for _ in range(3):
    g.stream_copy_dev(b, a, nb)
torch.cuda.synchronize()
g.timing(True)
g.timing_read("stream_copy")
for _ in range(10):
    g.stream_copy_dev(b, a, nb)
torch.cuda.synchronize()
ms, n = g.timing_read("stream_copy")
assert torch.equal(a[:1 << 20], b[:1 << 20])
print(os.path.basename(sys.argv[1]) if len(sys.argv) > 1 else "libnavgpu.so",
      "copy GB/s (read + write):", round(2 * nb / (ms / n * 1e-3) / 1e9, 1))
