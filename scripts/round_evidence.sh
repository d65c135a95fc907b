#!/bin/bash
# Round evidence in one gpurun session (outputs under gpurun_out/<tag>/):
#   GPU tests -> smoke -> K3 kernel trace -> FETCH_SIZE / WRITE_SIZE passes
#   (separate --pmc runs, no trace domains) -> traffic json -> K3 bench line
#   (traffic + CPU baseline) -> K2, K4, K5 (exact, fast) bench lines.
# A crash/abort/timeout ends the script.
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export NAVSLAM_QUIET=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
step() {  # step <name> <timeout> cmd...
  local name=$1 tmo=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -n 2 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
step pytest 900 python3 -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic-json"
step trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH --json-out "$OUT/bench_traced.json"
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 $BENCH
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 $BENCH
F=$(find "$OUT/pmc_fetch" -name "*counter_collection.csv" | head -1)
W=$(find "$OUT/pmc_write" -name "*counter_collection.csv" | head -1)
step traffic 120 python3 scripts/traffic_json.py "$F" "$W" "$OUT/traffic_k3.json" "$TAG"
step bench 600 python3 bench.py --traffic-json "$OUT/traffic_k3.json" --json-out "$OUT/bench_k3.json"
step bench_k2 300 python3 bench.py --workload k2 --steps 10 --json-out "$OUT/bench_k2.json"
step bench_k4 400 python3 bench.py --workload k4 --steps 3 --warmup 1 --json-out "$OUT/bench_k4.json"
step bench_k5 400 python3 bench.py --workload k5 --steps 30 --warmup 2 --json-out "$OUT/bench_k5.json"
step bench_k5_fast 400 python3 bench.py --workload k5 --k5-mode fast --steps 30 --warmup 2 --json-out "$OUT/bench_k5_fast.json"
step trace_k5 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_k5" -o run --output-format csv -- python3 bench.py --workload k5 --k5-mode fast --steps 20 --warmup 2 --no-cpu-baseline
echo done
