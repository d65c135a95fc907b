#!/bin/bash
# r3 per-row iteration: the GPU test suite (TESTS filter, default all), then
# K2 (f64 and integer-mm) and K5 fast bench lines.
TAG=${1:-r}; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "${TESTS:-gpu or not gpu}" > "$OUT/pytest.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
run() {  # run <name> <timeout> bench args...
  local name=$1 tmo=$2; shift 2
  timeout -k 10 "$tmo" python3 bench.py "$@" --json-out "$OUT/$name.json" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-400
  if fatal $rc; then exit $rc; fi
}
run k2 300 --workload k2 --steps 10 --no-cpu-baseline
run k2i 300 --workload k2 --integer-mm --steps 10 --no-cpu-baseline
run k5f 400 --workload k5 --k5-mode fast --steps 30 --warmup 2 --no-cpu-baseline
