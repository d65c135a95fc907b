#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 TMPDIR=/tmp
V=nav-slam_amd/lib/variants
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
  --timeout-method thread -k knn > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest: $(tail -n 1 "$OUT/pytest.log")"; [ $rc -ne 0 ] && exit $rc
for v in "1:" "2:" "2:$V/libnavgpu_a4.so"; do
  m=${v%%:*}; l=${v#*:}
  NAVGPU_KNN_STATS=1 NAVGPU_KNN_MODE=$m timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 ${l:+--lib $l} > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
  echo "probe $v: $(cat "$OUT/probe.json")"
done
NAVGPU_KNN_MODE=2 timeout -k 10 120 python3 scripts/knng_timeline.py --lib $V/libnavgpu_stamps.so > "$OUT/tl.json" 2> "$OUT/tl.err" || { tail -3 "$OUT/tl.err"; exit 1; }
echo "timeline: $(cat "$OUT/tl.json")"
NAVGPU_KNN_MODE=2 bash scripts/pmc_probe.sh "$1/pmc2" | grep -v "^pmc\|copyBuffer"
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_KNN_MODE=1" "NAVGPU_KNN_MODE=2"
