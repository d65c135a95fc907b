#!/bin/bash
# r4: restored k_knnw + f32 screen counters + K2i tie-pass phases
TAG=${1:-r4s6}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "knn or pair or smoke or rows or screen" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
ST=nav-slam_amd/lib/var_st/libnavgpu_st.so
for i in "" "--integer"; do for f in 1 0; do
  NAVGPU_SCREEN_F32=$f timeout -k 10 120 python3 scripts/rows_match_probe.py --lib $ST $i > "$OUT/rmp.json" 2>&1 || { tail -3 "$OUT/rmp.json"; exit 1; }
  echo "f32=$f $i $(tail -n 1 $OUT/rmp.json)"
done; done
for m in 1 0; do
  NAVGPU_KNN_MODE=$m timeout -k 10 180 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline \
    --no-stream-copy --json-out "$OUT/k3_$m.json" > "$OUT/k3_$m.log" 2>&1 || { tail -5 "$OUT/k3_$m.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/k3_$m.json')); print('k3 mode $m', d['value'], d['ms_per_step'], d.get('kernel_us_isolated'))"
done
