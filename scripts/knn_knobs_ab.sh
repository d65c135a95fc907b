#!/bin/bash
# K3 k_knnw knobs: grid occupancy / x slicing (env), records per wave and
# register budget (variant builds); knn_probe query_us / build_us
TAG=${1:-knn_knobs}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1 NAVGPU_KNN_STATS=1
V=nav-slam_amd/lib/variants
p() {  # p <label> <lib> [VAR=value ...]
  local label=$1 lib=$2; shift 2
  env "$@" timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 --lib $lib > "$OUT/p.json" 2>&1 || { tail -3 "$OUT/p.json"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/p.json').read().strip().splitlines()[-1]); print('$label', round(d['query_us'],1), round(d['build_us'],1), d['slow_lanes'])"
}
for r in 1 2; do
  p base $V/libnavgpu_base.so
  p occ4 $V/libnavgpu_base.so NAVGPU_KNN_OCC=4
  p occ6 $V/libnavgpu_base.so NAVGPU_KNN_OCC=6
  p sx3 $V/libnavgpu_base.so NAVGPU_KNN_SX=3
  p sx5 $V/libnavgpu_base.so NAVGPU_KNN_SX=5
  p r640 $V/libnavgpu_r640.so
  p r960 $V/libnavgpu_r960.so
  p m4 $V/libnavgpu_m4.so
done
