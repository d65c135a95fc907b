#!/bin/bash
# k-NN A/B probes (scripts/knn_ab.sh without the tests) + the SQ counter passes
TAG=${1:-abp}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 NAVGPU_KNN_STATS=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for lib in "" nav-slam_amd/lib/variants/*.so; do
  timeout -k 10 120 python3 scripts/knn_probe.py --occ ${OCC:-5} --reps 20 ${lib:+--lib $lib} >> "$OUT/probe.log" 2>&1; rc=$?
  echo "probe $lib rc=$rc"; if fatal $rc; then exit $rc; fi
done
grep '^{' "$OUT/probe.log"
bash scripts/pmc_sq.sh $TAG/sq
