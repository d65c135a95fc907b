#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
  --timeout-method thread -k knn > "$OUT/pytest.log" 2>&1; rc=$?
tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
NAVGPU_KNN_STATS=1 timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
echo "probe: $(cat "$OUT/probe.json")"
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 3 "NAVGPU_KNN_MODE=2" "NAVGPU_KNN_MODE=1" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_fat.so" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/tr_bench" -o run --output-format csv -- \
  python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-stream-copy --json-out "$OUT/tr_bench.json" \
  > "$OUT/tr_bench.log" 2>&1 || { tail "$OUT/tr_bench.log"; exit 1; }
