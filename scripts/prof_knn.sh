#!/bin/bash
# kernel trace + a few PMC passes of the k-NN probe
OUT=gpurun_out/${1:-profk}; mkdir -p "$OUT"; shift
export TMPDIR=/tmp NAVGPU_KNN_OCC=${OCC:-5}
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 scripts/knn_probe.py --reps 5 > "$OUT/trace.log" 2>&1; rc=$?; echo "trace rc=$rc"; fatal $rc && exit $rc
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d "$OUT/pmc$i" -o run --output-format csv -- python3 scripts/knn_probe.py --reps 2 > "$OUT/pmc$i.log" 2>&1; rc=$?; echo "pmc$i rc=$rc"; fatal $rc && exit $rc
done
echo done
