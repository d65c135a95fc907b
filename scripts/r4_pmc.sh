#!/bin/bash
# r4: SQ counter passes of the K3 query pass under NAVGPU_KNN_MODE 0 and 1,
# then knn_probe over the variant libraries
TAG=${1:-r4pmc}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 NAVGPU_KNN_STATS=1 PYTHONUNBUFFERED=1 TMPDIR=/tmp
for m in 0 1; do
  NAVGPU_KNN_MODE=$m bash scripts/pmc_sq.sh "$TAG/sq_m$m" > "$OUT/sq_m$m.txt" 2>&1 || { cat "$OUT/sq_m$m.txt"; exit 1; }
  echo "== mode $m"; grep -A3 "pmc_" "$OUT/sq_m$m.txt" | grep "k_knn" 
done
for lib in nav-slam_amd/lib/variants/*.so; do
  NAVGPU_KNN_MODE=1 timeout -k 10 120 python3 scripts/knn_probe.py --occ 5 --reps 20 --lib $lib > "$OUT/probe.json" 2>&1 || exit 1
  echo "$lib $(tail -1 "$OUT/probe.json")"
done
