#!/bin/bash
# r4: k-NN GPU tests, then the variant probe A/B, then the bench of the default
TAG=${1:-r4s2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 ${PYT_LIMIT:-400} python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-knn or pair or smoke}" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
bash scripts/r4_var.sh "$TAG/v" ${ROUNDS:-2} || exit $?
for m in 1 0; do
  NAVGPU_KNN_MODE=$m timeout -k 10 180 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline \
    --no-stream-copy --json-out "$OUT/bench_$m.json" > "$OUT/bench_$m.log" 2>&1 || { tail -5 "$OUT/bench_$m.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$m.json')); print('bench mode=$m', d['value'], d['ms_per_step'], d.get('kernel_us_isolated'))"
done
