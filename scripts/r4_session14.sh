#!/bin/bash
# r4: K3 bench A/B: sx 4 vs 3, MINW 3 vs 4 (variant), interleaved rounds
TAG=${1:-r4s14}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
V=nav-slam_amd/lib/variants
b() {  # b <name> "<VAR=value ...>"
  env $2 timeout -k 10 180 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline \
    --no-stream-copy --json-out "$OUT/$1.json" > "$OUT/$1.log" 2>&1 || { tail -5 "$OUT/$1.log"; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.json')); print('$1', d['value'], d['ms_per_step'], d.get('kernel_us_isolated'))"
}
for r in 1 2 3; do
  b sx4 "" || exit 1
  b sx3 "NAVGPU_KNN_SX=3" || exit 1
  b sx3_m4 "NAVGPU_KNN_SX=3 NAVGPU_LIB=$V/libnavgpu_m4.so" || exit 1
done
