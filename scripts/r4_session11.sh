#!/bin/bash
# r4: f32 screen with the band fallback: row tests, then K4 / K2 f32 vs f64
TAG=${1:-r4s11}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "rows or screen or lazy or smoke or kd or shim" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
ST=nav-slam_amd/lib/var_st/libnavgpu_st.so
NAVGPU_SCREEN_F32=1 timeout -k 10 120 python3 scripts/rows_match_probe.py --lib $ST > "$OUT/rmp.json" 2>&1 || { tail -3 "$OUT/rmp.json"; exit 1; }
echo "stamps f32: $(tail -n 1 $OUT/rmp.json | cut -c1-400)"
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
echo "== k_knnw waves per workgroup"; VDIR=nav-slam_amd/lib/variants bash scripts/r4_var.sh "$TAG/vw" 2 || exit $?
for r in 1 2; do for l in st st0; do
  timeout -k 10 120 python3 scripts/rows_probe.py --integer --lib nav-slam_amd/lib/var_st/libnavgpu_$l.so \
    > "$OUT/rp_$l.json" 2>&1 || { tail -3 "$OUT/rp_$l.json"; exit 1; }
  echo "$l $(tail -n 1 $OUT/rp_$l.json | cut -c1-300)"
done; done
b k2i "" "--workload k2 --integer-mm" || exit 1
b k4i "" "--workload k4 --integer-mm" || exit 1
