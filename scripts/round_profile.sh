#!/bin/bash
# Round evidence in one gpurun session: GPU tests -> smoke -> rocprofv3 kernel
# trace of the bench -> FETCH_SIZE and WRITE_SIZE passes (separate, no trace
# domains) -> traffic per step -> bench line with roofline.traffic + CPU
# baseline -> K2 bench. A crash/abort/timeout ends the script.
# usage: scripts/round_profile.sh <tag>   (outputs under gpurun_out/<tag>/)
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
  tail -n 3 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
[ -n "$SKIP_BUILD" ] || step build 900 python3 -c "import __graft_entry__ as g; g.build()"
step pytest 1500 python3 -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic-json"
step trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $BENCH --json-out "$OUT/bench_traced.json"
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 $BENCH
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 $BENCH
F=$(find "$OUT/pmc_fetch" -name "*counter_collection.csv" | head -1)
W=$(find "$OUT/pmc_write" -name "*counter_collection.csv" | head -1)
step traffic 120 python3 scripts/traffic_json.py "$F" "$W" "$OUT/traffic_k3.json" "$TAG"
step bench 600 python3 bench.py --traffic-json "$OUT/traffic_k3.json" --json-out "$OUT/bench.json"
step bench_inflight1 300 python3 bench.py --inflight 1 --no-cpu-baseline --traffic-json "$OUT/traffic_k3.json" --json-out "$OUT/bench_inflight1.json"
step bench_k2 300 python3 bench.py --workload k2 --steps 10 --json-out "$OUT/bench_k2.json"
step bench_k4 300 python3 bench.py --workload k4 --steps 3 --warmup 1 --json-out "$OUT/bench_k4.json"
step trace_k4 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_k4" -o run --output-format csv -- python3 bench.py --workload k4 --steps 3 --warmup 1 --no-cpu-baseline
echo done
