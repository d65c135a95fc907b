#!/bin/bash
# r5 session b: k-NN tests, probe A/B, SQ counters of both query passes
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
  --timeout-method thread -k knn > "$OUT/pytest.log" 2>&1; rc=$?
tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for m in 1 2 1 2; do
  NAVGPU_KNN_STATS=1 NAVGPU_KNN_MODE=$m timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 \
    > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
  echo "mode $m: $(cat "$OUT/probe.json")"
done
NAVGPU_KNN_MODE=2 bash scripts/pmc_sq.sh "$1/sq2" || exit 1
NAVGPU_KNN_MODE=1 bash scripts/pmc_sq.sh "$1/sq1" || exit 1
