"""Cross-check of a K3 bench line against the rocprofv3 kernel trace of the
same run: per launch of the query pass (k_knnw<K> or k_knng<K>), the summed durations of the index build
kernels, of the query-stage kernels and of the curvature, beside the line's
HIP-event kernel_us (their span on the context's stream).

usage: trace_check.py KERNEL_STATS_CSV BENCH_JSON OUT_JSON"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import BUILD_KERNELS, QUERY_KERNELS, QUERY_MAIN  # noqa: E402

stats, line, out = sys.argv[1:4]
rows = list(csv.DictReader(open(stats)))
b = json.load(open(line))
launches = sum(int(r["Calls"]) for r in rows if any(m in r["Name"] for m in QUERY_MAIN))


def per_launch(keys):
    ns = sum(float(r["TotalDurationNs"]) for r in rows if any(k in r["Name"] for k in keys))
    return round(ns / max(launches, 1) / 1e3, 2)


main = [r for r in rows if any(m in r["Name"] for m in QUERY_MAIN)]
rec = {"launches": launches,
       # the dominant kernel alone (bench.py quotes it as the trace basis of
       # its roofline beside the HIP-event span)
       "main_kernel": main[0]["Name"] if main else None,
       "main_avg_us": (round(sum(float(r["TotalDurationNs"]) for r in main) / max(launches, 1) / 1e3, 2)
                       if main else None),
       "k": b["config"].get("k"), "points_per_cloud": b["config"].get("points_per_cloud"),
       "knn_mode": b["config"].get("knn_mode"),
       "trace_us": {"knn_build": per_launch(BUILD_KERNELS),
                    "knn_query": per_launch(QUERY_KERNELS),
                    "curvature": per_launch(("k_curvature",))},
       "line_kernel_us": b.get("kernel_us"),
       "pairs_in_flight": b["config"].get("pairs_in_flight")}
rec["ratio_line_over_trace"] = {k: round(b["kernel_us"][k] / v, 4)
                                for k, v in rec["trace_us"].items() if v and k in b["kernel_us"]}
with open(out, "w") as f:
    json.dump(rec, f, indent=1)
print(json.dumps(rec))
