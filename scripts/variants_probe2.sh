#!/bin/bash
# variants x occupancies, each probe repeated; order given by LIBS/OCCS
OUT=gpurun_out/${1:-var}; mkdir -p "$OUT"
for rep in ${REPS:-1 2}; do
for lib in ${LIBS}; do
  for occ in ${OCCS:-5}; do
    NAVGPU_KNN_OCC=$occ timeout -k 10 200 python3 scripts/knn_probe.py --occ $occ --lib nav-slam_amd/lib/variants/libnavgpu_$lib.so --reps 10 > "$OUT/p.log" 2>&1; rc=$?
    echo "rep=$rep $lib occ=$occ rc=$rc $(grep -o '"query_us": [0-9.]*' "$OUT/p.log")"
    if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  done
done
done
