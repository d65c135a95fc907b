#!/bin/bash
# Per-kernel isolated durations of the K3 k-NN (knn_probe.py, one pair at a time)
# for several library builds: r6_trace_ab.sh TAG label:lib.so ...
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for spec in "$@"; do
  label=${spec%%:*}; lib=${spec#*:}
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/$label" -o run --output-format csv -- python3 scripts/knn_probe.py --occ 5 --reps 10 ${lib:+--lib $lib} > "$OUT/$label.log" 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -3 "$OUT/$label.log"; exit $rc; fi
  python3 scripts/kstats.py "$label" "$(find "$OUT/$label" -name '*kernel_stats.csv' | head -1)"
done
