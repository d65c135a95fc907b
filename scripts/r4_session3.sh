#!/bin/bash
# r4: the whole GPU suite, then the K3 / K4 / K5 bench lines the round's
# changes move (k_knnw vs k_knn, f32 screen on/off, K5 host trees on/off)
TAG=${1:-r4s3}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 ${PYT_LIMIT:-700} python3 -u -m pytest tests -m gpu -x -v --timeout 120 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
fi
b() {  # b <name> "<VAR=value ...>" "<bench.py arguments>"
  env $2 timeout -k 10 180 python3 bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline \
    --no-stream-copy $3 --json-out "$OUT/$1.json" > "$OUT/$1.log" 2>&1 || { tail -5 "$OUT/$1.log"; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.json')); print('$1', d['value'], d['unit'], d['ms_per_step'], d.get('kernel_us_isolated'))"
}
[ -n "$NO_BENCH" ] && exit 0
b k3_w "NAVGPU_KNN_MODE=1" "" || exit 1
b k3_t "NAVGPU_KNN_MODE=0" "" || exit 1
b k4_f32 "NAVGPU_SCREEN_F32=1" "--workload k4" || exit 1
b k4_f64 "NAVGPU_SCREEN_F32=0" "--workload k4" || exit 1
b k2_f32 "NAVGPU_SCREEN_F32=1" "--workload k2" || exit 1
b k2_f64 "NAVGPU_SCREEN_F32=0" "--workload k2" || exit 1
b k5f_lazy "NAVSLAM_HOST_TREES=0" "--workload k5 --k5-mode fast" || exit 1
b k5f_trees "NAVSLAM_HOST_TREES=1" "--workload k5 --k5-mode fast" || exit 1
b k2i "" "--workload k2 --integer-mm" || exit 1
b k2i_nth1 "NAVGPU_LIB=nav-slam_amd/lib/var_nth/libnavgpu_nth1.so" "--workload k2 --integer-mm" || exit 1
b k4i "" "--workload k4 --integer-mm" || exit 1
b k2i_t128 "NAVGPU_LIB=nav-slam_amd/lib/var_nth/libnavgpu_t128.so" "--workload k2 --integer-mm" || exit 1
b k2i_l256 "NAVGPU_LIB=nav-slam_amd/lib/var_nth/libnavgpu_l256.so" "--workload k2 --integer-mm" || exit 1
