#!/bin/bash
# full GPU test suite + smoke, then the per-row bench lines with CPU legs and
# kernel traces (K2, K4)
TAG=${1:-full}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
step() {  # step <name> <timeout> cmd...
  local name=$1 tmo=$2; shift 2
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  if fatal $rc; then echo "FATAL in $name"; exit $rc; fi
  return 0
}
step pytest 900 python3 -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_k2 600 python3 bench.py --workload k2 --steps 20 --json-out "$OUT/bench_k2.json"
step bench_k4 600 python3 bench.py --workload k4 --steps 5 --warmup 2 --json-out "$OUT/bench_k4.json"
step trace_k2 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_k2" -o run --output-format csv -- python3 bench.py --workload k2 --steps 20 --no-cpu-baseline
step trace_k4 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_k4" -o run --output-format csv -- python3 bench.py --workload k4 --steps 5 --warmup 2 --no-cpu-baseline
