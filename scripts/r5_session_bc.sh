#!/bin/bash
# K3 grid geometry sweep under k_knng: targets per h^3 and x slices
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
for r in 1 2 3; do
  for v in "NAVGPU_KNN_OCC=5" "NAVGPU_KNN_OCC=4" "NAVGPU_KNN_OCC=3.5" "NAVGPU_KNN_OCC=3" "NAVGPU_KNN_OCC=4.5"; do
    env $v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-traffic-json --no-stream-copy --json-out "$OUT/k3.json" > "$OUT/k3.log" 2>&1 || { tail "$OUT/k3.log"; exit 1; }
    python3 scripts/k3_line_summary.py "$v" "$OUT/k3.json"
  done
done
