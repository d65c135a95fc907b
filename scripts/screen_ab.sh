#!/bin/bash
# The f32 screen with fused curvature: row tests, then K4 / K2 fused vs
# unfused vs f64, K4 with 256-thread screen blocks
TAG=${1:-screen_ab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "rows or screen or lazy or smoke or shim or bench" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
b() {  # b <name> "<VAR=value ...>" "<bench.py arguments>"
  env $2 timeout -k 10 180 python3 bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline \
    --no-stream-copy $3 --json-out "$OUT/$1.json" > "$OUT/$1.log" 2>&1 || { tail -5 "$OUT/$1.log"; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.json')); print('$1', d['value'], d['unit'], d['ms_per_step'], d.get('kernel_us'))"
}
for r in 1 2; do
  b k4_fused "" "--workload k4" || exit 1
  b k4_unfused "NAVGPU_SCREEN_FUSE=0" "--workload k4" || exit 1
  b k4_f64 "NAVGPU_SCREEN_F32=0" "--workload k4" || exit 1
  b k4_fused_nt256 "NAVGPU_SCREEN_NT=256" "--workload k4" || exit 1
  b k2_fused "" "--workload k2" || exit 1
  b k2_unfused "NAVGPU_SCREEN_FUSE=0" "--workload k2" || exit 1
done
