#!/bin/bash
# k-NN probe over k_knn grid sizes (blocks per XCD)
OUT=gpurun_out/${1:-swb}; mkdir -p "$OUT"
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for nb in ${NBS:-96 128 160 192 256 320}; do
  NAVGPU_KNN_BLOCKS=$nb timeout -k 10 300 python3 scripts/knn_probe.py --occ ${OCC:-5} > "$OUT/nb$nb.log" 2>&1; rc=$?
  echo "nb=$nb rc=$rc $(grep query_us "$OUT/nb$nb.log")"; if fatal $rc; then exit $rc; fi
done
