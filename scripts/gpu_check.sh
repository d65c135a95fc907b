#!/bin/bash
# One gpurun session: GPU tests -> smoke -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/abort/timeout (rc >= 124 or
# a signal) ends the script, plain test failures (rc 1) do not.
# usage: scripts/gpu_check.sh [tag] [pytest-args...]
TAG=${1:-r1}; shift
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
  tail -n 5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
[ -n "$SKIP_BUILD" ] || step build 600 python3 -c "import __graft_entry__ as g; g.build()"
step pytest 1500 python3 -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread "$@"
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py --json-out "$OUT/bench.json"
step bench_k2 300 python3 bench.py --workload k2 --steps 10 --json-out "$OUT/bench_k2.json"
export TMPDIR=/tmp
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
echo done
