#!/bin/bash
# Round evidence in one gpurun session (outputs under gpurun_out/<tag>/):
#   GPU tests -> smoke -> K3 kernel trace -> per workload (K3, K2, K2 integer-mm,
#   K4, K4 integer-mm, K5 fast) a FETCH_SIZE and a WRITE_SIZE pass (separate
#   --pmc runs, no trace domains) -> traffic_<w>.json -> the bench lines, each
#   quoting its own traffic json (K3 also with the CPU baseline).
# A crash/abort/timeout ends the script. SKIP_TESTS=1 skips pytest + smoke.
# PARTS (default "tests k3 pmc bench") picks the sections, so the session can
# be split over several gpurun calls.
TAG=${1:-r3}
PARTS=${PARTS:-tests k3 pmc bench}
part() { case " $PARTS " in *" $1 "*) return 0;; esac; return 1; }
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
step() {  # step <name> <timeout> cmd...
  local name=$1 tmo=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -n 2 "$OUT/$name.log" | cut -c1-300
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return 0
}
if [ -z "$SKIP_TESTS" ] && part tests; then
  step pytest 900 python3 -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-traffic-json --no-stream-copy"
if part k3; then
step trace_k3 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_k3" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 $Q --json-out "$OUT/bench_k3_traced.json"
# one pair at a time: the trace's per-launch kernel sums and the line's HIP
# events time the same isolated kernels
step trace_k3_iso 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_k3_iso" -o run --output-format csv -- python3 bench.py --inflight 1 --steps 20 --warmup 3 $Q --json-out "$OUT/bench_k3_iso_traced.json"
step trace_check 60 python3 scripts/trace_check.py "$(find "$OUT/trace_k3_iso" -name "*kernel_stats.csv" | head -1)" "$OUT/bench_k3_iso_traced.json" "$OUT/trace_check_k3.json"
# the bench lines below quote it (bench.py load_trace); commit it afterwards
cp "$OUT/trace_check_k3.json" profiles/trace_k3.json
fi
pmc() {  # pmc <w> <traffic args> -- <bench args>
  local w=$1; shift
  local targs=()
  while [ "$1" != "--" ]; do targs+=("$1"); shift; done; shift
  step pmc_fetch_$w 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$w" -o run --output-format csv -- python3 bench.py "$@" $Q
  step pmc_write_$w 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$w" -o run --output-format csv -- python3 bench.py "$@" $Q
  local F W
  F=$(find "$OUT/pmc_fetch_$w" -name "*counter_collection.csv" | head -1)
  W=$(find "$OUT/pmc_write_$w" -name "*counter_collection.csv" | head -1)
  step traffic_$w 120 python3 scripts/traffic_json.py "$F" "$W" "$OUT/traffic_$w.json" "$TAG" --workload "$w" "${targs[@]}" --src "python3 bench.py $*"
}
if part k3; then
pmc k3 -- --steps 20 --warmup 3
# the query pass's instruction mix, one pair at a time (its own --pmc run)
step pmc_sq_k3 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$OUT/pmc_sq_k3" -o run --output-format csv -- python3 bench.py --inflight 1 --steps 10 --warmup 2 $Q
fi
if part pmc; then
pmc k2 --points 262144 --pairs 1 -- --workload k2 --steps 10
pmc k2i --points 262144 --pairs 1 -- --workload k2 --integer-mm --steps 10
pmc k4 --points 262144 --pairs 256 -- --workload k4 --steps 2 --warmup 1
pmc k4i --points 262144 --pairs 256 -- --workload k4 --integer-mm --steps 2 --warmup 1
pmc k5f --points 262144 -- --workload k5 --k5-mode fast --steps 20 --warmup 2
NAVSLAM_HOST_TREES=0 pmc k5fl --points 262144 -- --workload k5 --k5-mode fast --steps 20 --warmup 2
fi
if part bench; then
# a traffic json made earlier in this session, else the committed one
tj() { if [ -f "$OUT/traffic_$1.json" ]; then echo "$OUT/traffic_$1.json"; else echo "profiles/traffic_$1.json"; fi; }
step bench_k3 600 python3 bench.py --traffic-json "$(tj k3)" --json-out "$OUT/bench_k3.json"
step bench_k3_inflight1 300 python3 bench.py --inflight 1 --no-cpu-baseline --traffic-json "$(tj k3)" --json-out "$OUT/bench_k3_inflight1.json"
step bench_k2 300 python3 bench.py --workload k2 --steps 100 --traffic-json "$(tj k2)" --json-out "$OUT/bench_k2.json"
step bench_k2i 300 python3 bench.py --workload k2 --integer-mm --steps 100 --traffic-json "$(tj k2i)" --json-out "$OUT/bench_k2i.json"
step bench_k4 400 python3 bench.py --workload k4 --steps 10 --warmup 2 --traffic-json "$(tj k4)" --json-out "$OUT/bench_k4.json"
step bench_k4i 400 python3 bench.py --workload k4 --integer-mm --steps 10 --warmup 2 --traffic-json "$(tj k4i)" --json-out "$OUT/bench_k4i.json"
step bench_k5 400 python3 bench.py --workload k5 --steps 30 --warmup 2 --json-out "$OUT/bench_k5.json"
step bench_k5_fast 400 python3 bench.py --workload k5 --k5-mode fast --steps 30 --warmup 2 --traffic-json "$(tj k5f)" --json-out "$OUT/bench_k5_fast.json"
NAVSLAM_HOST_TREES=0 step bench_k5_fast_lazy 400 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --traffic-json "$(tj k5fl)" --json-out "$OUT/bench_k5_fast_lazy.json"
NAVSLAM_HOST_TREES=0 step bench_k5_fast_lazy_10k 600 python3 bench.py --workload k5 --k5-mode fast --steps 9990 --warmup 10 --traffic-json "$(tj k5fl)" --no-cpu-baseline --json-out "$OUT/bench_k5_fast_lazy_10k.json"
step trace_k5 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace_k5" -o run --output-format csv -- python3 bench.py --workload k5 --k5-mode fast --steps 20 --warmup 2 --no-cpu-baseline --no-traffic-json
fi
echo done
