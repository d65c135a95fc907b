#!/bin/bash
# per-row path session: row parity tests, then K2 / K4 bench lines (no CPU legs)
TAG=${1:-rows}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
PYTHONUNBUFFERED=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread -k "${KSEL:-rows}" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 5 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --workload k2 --steps 20 --no-cpu-baseline --json-out "$OUT/bench_k2.json" > "$OUT/bench_k2.log" 2>&1; rc=$?
echo "k2 rc=$rc"; tail -n 1 "$OUT/bench_k2.log" | cut -c1-600; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python3 bench.py --workload k4 --steps 5 --warmup 2 --no-cpu-baseline --json-out "$OUT/bench_k4.json" > "$OUT/bench_k4.log" 2>&1; rc=$?
echo "k4 rc=$rc"; tail -n 1 "$OUT/bench_k4.log" | cut -c1-600; if fatal $rc; then exit $rc; fi
if [ -n "$TRACE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_k2" -o run --output-format csv -- python3 bench.py --workload k2 --steps 20 --no-cpu-baseline > "$OUT/trace_k2.log" 2>&1; echo "trace rc=$?"
fi
