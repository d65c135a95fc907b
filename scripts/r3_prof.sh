#!/bin/bash
# r3: kernel trace (+ stats) of the isolated K3 k-NN call (knn_sweep.py), and
# optionally FETCH_SIZE / WRITE_SIZE passes (PMC=1), each its own run
TAG=${1:-p}; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1 TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
CFG=${CFG:-SX=4}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 scripts/knn_sweep.py --reps 10 "$CFG" > "$OUT/trace.log" 2>&1; rc=$?
echo "trace rc=$rc"; if fatal $rc; then exit $rc; fi
S=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
python3 - "$S" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print("%-60s calls=%5s avg_us=%8.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
if [ -n "$PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- python3 scripts/knn_sweep.py --reps 3 "$CFG" > "$OUT/pmc_$c.log" 2>&1; rc=$?
    echo "pmc $c rc=$rc"; if fatal $rc; then exit $rc; fi
  done
  python3 scripts/pmc_summary.py "$OUT" all > "$OUT/pmc_summary.txt" 2>&1; cat "$OUT/pmc_summary.txt" | head -30
fi
