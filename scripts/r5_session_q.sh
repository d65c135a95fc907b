#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
bash scripts/r5_session_p.sh "$1/k5" || exit 1
V=nav-slam_amd/lib/variants
for r in 1 2; do
for v in "" ntq nto ntb; do
  l=${v:+$V/libnavgpu_$v.so}
  NAVGPU_KNN_MODE=2 timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 ${l:+--lib $l} > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
  echo "probe ${v:-base}: $(python3 -c "import json; d=json.load(open('$OUT/probe.json')); print(round(d['query_us'],1), round(d['build_us'],1), d['slow_lanes'])")"
done
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_KNN_MODE=2" "NAVGPU_KNN_MODE=2 NAVGPU_LIB=$V/libnavgpu_ntb.so" "NAVGPU_KNN_MODE=2 NAVGPU_LIB=$V/libnavgpu_nto.so"
