#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 TMPDIR=/tmp
V=nav-slam_amd/lib/variants
NAVGPU_KNN_MODE=2 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
  --timeout-method thread -k "knn and mode2" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest: $(tail -n 1 "$OUT/pytest.log")"; [ $rc -ne 0 ] && exit $rc
for v in "1:" "2:" "2:$V/libnavgpu_nb1k.so" "2:$V/libnavgpu_nb4k.so"; do
  m=${v%%:*}; l=${v#*:}
  NAVGPU_KNN_MODE=$m timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 ${l:+--lib $l} > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
  echo "probe $v: $(cat "$OUT/probe.json")"
done
NAVGPU_KNN_MODE=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/tr_iso" -o run --output-format csv -- \
  python3 scripts/knn_probe.py --reps 10 > "$OUT/tr_iso.log" 2>&1 || { tail "$OUT/tr_iso.log"; exit 1; }
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_KNN_MODE=1" "NAVGPU_KNN_MODE=2"
