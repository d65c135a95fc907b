#!/bin/bash
# r4: row-path tests, then K4 / K2 (f32 vs f64 screen), K2i / K4i (tie walks
# stop at the screen's minimum), K5 fast lazy
TAG=${1:-r4s8}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "rows or screen or lazy or shim or kd or smoke or k1" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
b() {  # b <name> "<VAR=value ...>" "<bench.py arguments>"
  env $2 timeout -k 10 180 python3 bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline \
    --no-stream-copy $3 --json-out "$OUT/$1.json" > "$OUT/$1.log" 2>&1 || { tail -5 "$OUT/$1.log"; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.json')); print('$1', d['value'], d['unit'], d['ms_per_step'], d.get('kernel_us'))"
}
for r in 1 2; do
  b k4_f32 "NAVGPU_SCREEN_F32=1" "--workload k4" || exit 1
  b k4_f64 "NAVGPU_SCREEN_F32=0" "--workload k4" || exit 1
  b k2_f32 "NAVGPU_SCREEN_F32=1" "--workload k2" || exit 1
  b k2_f64 "NAVGPU_SCREEN_F32=0" "--workload k2" || exit 1
done
b k2i "" "--workload k2 --integer-mm" || exit 1
b k4i "" "--workload k4 --integer-mm" || exit 1
b k5f_lazy "NAVSLAM_HOST_TREES=0" "--workload k5 --k5-mode fast" || exit 1
