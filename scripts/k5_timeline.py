"""Print one K5 frame's kernel + copy timeline from a rocprofv3 kernel/memory-copy
trace (csv): scripts/k5_timeline.py PROFDIR [prefix]"""
import csv
import re
import sys

d = sys.argv[1]
pre = sys.argv[2] if len(sys.argv) > 2 else "k5"


def nm(s):
    m = re.search(r"k_\w+|__amd_\w+", s)
    return m.group(0) if m else s[:30]


ev = []
for r in csv.DictReader(open(f"{d}/{pre}_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm(r["Kernel_Name"]), r.get("Stream_Id", "")))
for r in csv.DictReader(open(f"{d}/{pre}_memory_copy_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r["Direction"][12:], r["Stream_Id"]))
ev.sort()
ki = [i for i, e in enumerate(ev) if "rows_query" in e[2]]
mid = ki[len(ki) // 2]
w = ev[mid - 14:mid + 16]
t0, prev = w[0][0], None
print(f"{'start_us':>9} {'dur_us':>7} {'gap_us':>7}  stream event")
for s, e, n, q in w:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {((s - prev) / 1e3 if prev else 0):7.1f}  s{q} {n}")
    prev = max(prev or 0, e)
