"""Per-step HBM bytes of the K3 k-NN query stage and of the index build from
the FETCH_SIZE and WRITE_SIZE rocprofv3 passes of bench.py (or of
knn_sweep.py) -> a small JSON bench.py quotes as roofline.traffic and
roofline.build.traffic (the counters cannot run inside the timed bench)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import BUILD_KERNELS, QUERY_KERNELS, pmc_bytes  # noqa: E402

fetch_csv, write_csv, out, tag = sys.argv[1:5]
src = sys.argv[5] if len(sys.argv) > 5 else "python3 bench.py --steps 20 --warmup 3"
q = pmc_bytes([fetch_csv, write_csv], QUERY_KERNELS)
b = pmc_bytes([fetch_csv, write_csv], BUILD_KERNELS)
main = pmc_bytes([fetch_csv, write_csv], ("k_knn<",))
rec = {"workload": "k3", "k": 8, "points_per_cloud": 1048576,
       "bytes_per_step": q and q["bytes"], "build_bytes_per_step": b and b["bytes"],
       "query": q, "build": b, "k_knn_main": main,
       "kernels": {"query": list(QUERY_KERNELS), "build": list(BUILD_KERNELS)},
       "source": (f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of `{src}`, round "
                  f"tag {tag}; bytes = FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md "
                  "HBM section) + WRITE_SIZE, per launch of k_knn<8>; fetch_raw = FETCH_SIZE "
                  "as counted")}
with open(out, "w") as f:
    json.dump(rec, f, indent=1)
print(json.dumps(rec))
