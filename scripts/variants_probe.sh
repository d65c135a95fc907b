#!/bin/bash
OUT=gpurun_out/${1:-var}; mkdir -p "$OUT"
for lib in nav-slam_amd/lib/variants/*.so; do
  for occ in ${OCCS:-5}; do
    NAVGPU_KNN_OCC=$occ timeout -k 10 200 python3 scripts/knn_probe.py --occ $occ --lib $lib --reps 10 >> "$OUT/probe.log" 2>&1; rc=$?
    echo "$lib occ=$occ rc=$rc"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  done
done
grep occ "$OUT/probe.log"
