#!/bin/bash
# r4 k-NN session: the k-NN GPU tests under the default query pass, then an
# interleaved A/B of the query passes (NAVGPU_KNN_MODE 0 = k_knn block tiles,
# 1 = k_knnw wave chunks): knn_probe isolated times and the K3 bench step.
TAG=${1:-r4ab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 NAVGPU_KNN_STATS=1 PYTHONUNBUFFERED=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-knn}" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 5 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for m in ${MODES:-0 1}; do
    NAVGPU_KNN_MODE=$m timeout -k 10 120 python3 scripts/knn_probe.py --occ 5 --reps 20 > "$OUT/probe_$m.json" 2>&1; rc=$?
    echo "mode=$m round=$r $(cat "$OUT/probe_$m.json" | tail -1)"; fatal $rc && exit $rc
  done
done
for r in 1 2; do
  for m in ${MODES:-0 1}; do
    NAVGPU_KNN_MODE=$m timeout -k 10 180 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline \
      --no-stream-copy --json-out "$OUT/bench_$m.json" > "$OUT/bench_$m.log" 2>&1; rc=$?
    fatal $rc && { tail -5 "$OUT/bench_$m.log"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$OUT/bench_$m.json')); print('mode=$m round=$r', d['value'], d['ms_per_step'], d.get('kernel_us_isolated'))"
  done
done
