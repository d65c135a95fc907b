#!/bin/bash
# knn_probe over every variant library x NAVGPU_KNN_BLOCKS values (NBS)
OUT=gpurun_out/${1:-vnb}; mkdir -p "$OUT"
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for lib in nav-slam_amd/lib/variants/*.so; do
  for nb in ${NBS:-768}; do
    NAVGPU_KNN_BLOCKS=$nb timeout -k 10 120 python3 scripts/knn_probe.py --occ ${OCC:-5} --reps 20 --lib $lib > "$OUT/p.log" 2>&1; rc=$?
    echo "$(basename $lib) nb=$nb rc=$rc $(grep -o '"query_us": [0-9.]*' $OUT/p.log) $(grep -o '"slow_lanes": [0-9]*' $OUT/p.log)"
    if fatal $rc; then exit $rc; fi
  done
done
