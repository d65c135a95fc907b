#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 TMPDIR=/tmp
V=nav-slam_amd/lib/variants
for l in "" $V/libnavgpu_w4.so $V/libnavgpu_fatw4.so; do
  NAVGPU_KNN_STATS=1 timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 ${l:+--lib $l} > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
  echo "probe $l: $(cat "$OUT/probe.json")"
done
for l in stamps w4stamps; do
  timeout -k 10 120 python3 scripts/knng_timeline.py --lib $V/libnavgpu_$l.so > "$OUT/tl_$l.json" 2> "$OUT/tl.err" || { tail -3 "$OUT/tl.err"; exit 1; }
  echo "$l: $(cat "$OUT/tl_$l.json")"
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_KNN_MODE=1" "NAVGPU_LIB=$V/libnavgpu_w4.so" "NAVGPU_LIB=$V/libnavgpu_fatw4.so" "NAVGPU_LIB=$V/libnavgpu_fat.so"
