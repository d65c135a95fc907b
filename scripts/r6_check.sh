#!/bin/bash
# r6 quick check: selected GPU tests (-k expression $1) then the default bench line.
TAG=${TAG:-r6a}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$1" \
  > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 400 python3 bench.py ${BENCH_ARGS:---no-cpu-baseline} --json-out "$OUT/bench_k3.json" > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
python3 scripts/k3_line_summary.py "$TAG" "$OUT/bench_k3.json" || head -c 1500 "$OUT/bench_k3.json"
