#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 TMPDIR=/tmp
V=nav-slam_amd/lib/variants
for m in 3 2; do
  NAVGPU_KNN_MODE=$m timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
    --timeout-method thread -k knn > "$OUT/pytest_m$m.log" 2>&1; rc=$?
  echo "mode $m: $(tail -n 1 "$OUT/pytest_m$m.log")"; [ $rc -ne 0 ] && exit $rc
done
for m in 1 2 3; do
  NAVGPU_KNN_MODE=$m NAVGPU_KNN_STATS=1 timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
  echo "probe $m: $(cat "$OUT/probe.json")"
done
NAVGPU_KNN_MODE=3 timeout -k 10 120 python3 scripts/knng_timeline.py --lib $V/libnavgpu_stamps.so > "$OUT/tl.json" 2> "$OUT/tl.err" || { tail -3 "$OUT/tl.err"; exit 1; }
echo "timeline m3: $(cat "$OUT/tl.json")"
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_KNN_MODE=1" "NAVGPU_KNN_MODE=2" "NAVGPU_KNN_MODE=3"
