#!/bin/bash
# k-NN grid occupancy sweep: kernel times + slow-path counts per setting.
OUT=gpurun_out/${1:-sweep}; shift
mkdir -p "$OUT"
export NAVGPU_KNN_STATS=1
for occ in "$@"; do
  NAVGPU_KNN_OCC=$occ timeout -k 10 300 python3 scripts/knn_probe.py --occ "$occ" >> "$OUT/sweep.log" 2>&1
  rc=$?
  echo "occ=$occ rc=$rc" >> "$OUT/sweep.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
cat "$OUT/sweep.log"
