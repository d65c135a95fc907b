#!/bin/bash
# r4: screen phase stamps (f32 vs f64), then the persistent k_knnw grid sizes
TAG=${1:-r4s10}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
ST=nav-slam_amd/lib/var_st/libnavgpu_st.so
for r in 1 2; do for f in 1 0; do
  NAVGPU_SCREEN_F32=$f timeout -k 10 120 python3 scripts/rows_match_probe.py --lib $ST > "$OUT/rmp.json" 2>&1 || { tail -3 "$OUT/rmp.json"; exit 1; }
  echo "f32=$f $(tail -n 1 $OUT/rmp.json | cut -c1-600)"
done; done
bash scripts/r4_session9.sh "$TAG/p9"
