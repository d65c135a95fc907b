"""Summarise rocprofv3 kernel stats + counter CSVs under a gpurun_out dir."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    print("== kernel stats", f)
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:70]:70s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r["Dispatch_Id"])
    print("==", f)
    for k, v in agg.items():
        if "knn" in k or len(sys.argv) > 2:
            print("  ", k, {c: round(x / len(n[k])) for c, x in v.items()})
