"""One line of per-kernel average durations (us) from a rocprofv3 kernel_stats.csv:
python3 scripts/kstats.py LABEL run_kernel_stats.csv"""
import csv
import sys

rows = {}
for r in csv.DictReader(open(sys.argv[2])):
    n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    rows[n.split("(")[0]] = float(r["AverageNs"]) / 1e3
keep = sorted(k for k in rows if k.startswith("k_"))
build = sum(rows[k] for k in keep if k.startswith(("k_bbox", "k_bin", "k_nb")))
print(sys.argv[1], " ".join(f"{k}={rows[k]:.1f}" for k in keep), f"| build={build:.1f}")
