"""Per-step HBM bytes of the k-NN query stage from the FETCH_SIZE and
WRITE_SIZE rocprofv3 passes of bench.py -> a small JSON bench.py can quote
as roofline.traffic (the counters cannot run inside the timed bench)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import traffic_from_csv  # noqa: E402

fetch_csv, write_csv, out, tag = sys.argv[1:5]
t = traffic_from_csv([fetch_csv, write_csv], "k_knn")
rec = {"workload": "k3", "k": 8, "points_per_cloud": 1048576, "bytes_per_step": t,
       "kernels": "k_knn<8,false> + k_knn<8,true> + k_knn_slow<8>",
       "source": (f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of `python3 "
                  f"bench.py --steps 20 --warmup 3`, round tag {tag}; FETCH_SIZE x2 "
                  "(gfx950 correction, MI355X_MICROARCH.md HBM section) + WRITE_SIZE, "
                  "per launch of k_knn<8,false>")}
with open(out, "w") as f:
    json.dump(rec, f, indent=1)
print(json.dumps(rec))
