#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
  --timeout-method thread -k knn > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest: $(tail -n 1 "$OUT/pytest.log")"; [ $rc -ne 0 ] && exit $rc
for m in 1 2; do
  NAVGPU_KNN_STATS=1 NAVGPU_KNN_MODE=$m timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
  echo "probe $m: $(cat "$OUT/probe.json")"
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_KNN_MODE=1" "NAVGPU_KNN_MODE=2"
