"""Per-step HBM bytes from the FETCH_SIZE and WRITE_SIZE rocprofv3 passes of a
bench.py run -> profiles/traffic_<tag>.json, which bench.py quotes as
roofline.traffic (and, for K3, roofline.build.traffic): the counters cannot
run inside the timed bench.

usage: traffic_json.py FETCH_CSV WRITE_CSV OUT ROUND_TAG [--workload k3|k2|k2i|k4|k4i|k5|k5f|k5fl]
                       [--points N] [--pairs P] [--k K] [--src "command"]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import QUERY_MAIN, TRAFFIC_SETS, pmc_bytes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("fetch_csv")
ap.add_argument("write_csv")
ap.add_argument("out")
ap.add_argument("tag")
ap.add_argument("--workload", default="k3")
ap.add_argument("--points", type=int, default=1048576)
ap.add_argument("--pairs", type=int, default=1)
ap.add_argument("--k", type=int, default=8)
ap.add_argument("--src", default="python3 bench.py --steps 20 --warmup 3")
a = ap.parse_args()
paths = [a.fetch_csv, a.write_csv]
note = ("bytes = FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md HBM section) + "
        "WRITE_SIZE; fetch_raw = FETCH_SIZE as counted")
if a.workload == "k3":
    q = pmc_bytes(paths, *TRAFFIC_SETS["k3"])
    b = pmc_bytes(paths, *TRAFFIC_SETS["k3_build"])
    main = pmc_bytes(paths, QUERY_MAIN, QUERY_MAIN)
    rec = {"workload": "k3", "k": a.k, "points_per_cloud": a.points,
           "bytes_per_step": q and q["bytes"], "build_bytes_per_step": b and b["bytes"],
           "query": q, "build": b, "k_knn_main": main,
           "kernels": {"query": list(TRAFFIC_SETS["k3"][0]),
                       "build": list(TRAFFIC_SETS["k3_build"][0])},
           "per": "launch of the query pass k_knng<K> / k_knnw<K> (one per step)"}
else:
    key = "k5" if a.workload.startswith("k5") else "rows"
    kern, anchor = TRAFFIC_SETS[key]
    t = pmc_bytes(paths, kern, anchor)
    per_kernel = {k: pmc_bytes(paths, (k,), anchor) for k in kern}
    rec = {"workload": a.workload, "points_per_cloud": a.points,
           "bytes_per_step": t and t["bytes"], "total": t, "per_kernel": per_kernel,
           "kernels": list(kern), "per": f"launch of {anchor} (one per step)"}
    if key == "rows":
        rec["pairs_per_step"] = a.pairs
rec["source"] = (f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of `{a.src}`, round "
                 f"tag {a.tag}; " + note)
with open(a.out, "w") as f:
    json.dump(rec, f, indent=1)
print(json.dumps(rec))
