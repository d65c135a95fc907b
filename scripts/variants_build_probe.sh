#!/bin/bash
# variants: k-NN index build time (knn_build region) and query time
OUT=gpurun_out/${1:-vb}; mkdir -p "$OUT"
for lib in ${LIBS}; do
  NAVGPU_KNN_OCC=${OCC:-5} timeout -k 10 200 python3 scripts/knn_probe.py --lib nav-slam_amd/lib/variants/libnavgpu_$lib.so --reps 20 > "$OUT/p.log" 2>&1; rc=$?
  echo "$lib rc=$rc $(grep -o '"query_us": [0-9.]*, "build_us": [0-9.]*' "$OUT/p.log")"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
