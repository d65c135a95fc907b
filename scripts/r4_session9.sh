#!/bin/bash
# r4: persistent k_knnw grid sizes (NAVGPU_KNN_BLOCKS = workgroups per XCD)
# against the per-chunk launch, knn_probe query_us / build_us
TAG=${1:-r4s9}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1 NAVGPU_KNN_MODE=1
V=nav-slam_amd/lib/variants
p() {  # p <label> <lib> [blocks]
  NAVGPU_KNN_BLOCKS=${3:-0} timeout -k 10 120 python3 scripts/knn_probe.py --occ 5 --reps 20 --lib $2 > "$OUT/p.json" 2>&1 || { tail -3 "$OUT/p.json"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/p.json').read().strip().splitlines()[-1]); print('$1', round(d['query_us'],1), round(d['build_us'],1), d['slow_lanes'])"
}
for r in 1 2; do
  p cur $V/libnavgpu_cur.so
  p pers_api $V/libnavgpu_pers.so
  for b in 96 128 160 192 256; do p pers_$b $V/libnavgpu_pers.so $b; done
done
