#!/bin/bash
# GPU tests, then K5 stream lines: exact and fast modes (no CPU legs unless CPU=1)
TAG=${1:-k5}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
step() {
  local name=$1 tmo=$2; shift 2
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "FAILED in $name"; exit $rc; fi
}
CB=${CPU:+}; [ -z "$CPU" ] && CB=--no-cpu-baseline
[ -n "$SKIP_TESTS" ] || step pytest 900 python3 -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread ${PYTEST_K:+-k "$PYTEST_K"}
step k5_exact 900 python3 bench.py --workload k5 --k5-mode exact --steps ${EXACT_STEPS:-60} --warmup 3 $CB --json-out "$OUT/bench_k5_exact.json"
step k5_fast 900 python3 bench.py --workload k5 --k5-mode fast --steps ${FAST_STEPS:-300} --warmup 3 $CB --json-out "$OUT/bench_k5_fast.json"
