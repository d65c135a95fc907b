#!/bin/bash
# r4: quick A/B after the f32-screen setup rework: row tests, K4/K2 f32 vs
# f64, then the k_knnw probe (committed c47 vs persistent variants)
TAG=${1:-r4s5}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "rows or screen or lazy or smoke" > "$OUT/pytest.log" 2>&1; rc=$?
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
b k5f_lazy_prof "NAVSLAM_HOST_TREES=0 NAVSLAM_PROFILE=1" "--workload k5 --k5-mode fast" || exit 1
grep -i "navslam" "$OUT/k5f_lazy_prof.log" | head -8
for r in 1 2; do for l in st1 st2; do
  timeout -k 10 120 python3 scripts/rows_probe.py --integer --lib nav-slam_amd/lib/var_st/libnavgpu_$l.so \
    > "$OUT/rp_$l.json" 2>&1 || { tail -3 "$OUT/rp_$l.json"; exit 1; }
  tail -n 1 "$OUT/rp_$l.json" | cut -c1-400
done; done
echo "== k_knnw variants"; VDIR=nav-slam_amd/lib/variants bash scripts/r4_var.sh "$TAG/vw" 2 || exit $?
