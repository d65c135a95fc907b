#!/bin/bash
# r4: knn_probe over the variant libraries, interleaved rounds (query pass 1 = k_knnw)
OUT=gpurun_out/${1:-r4v}; ROUNDS=${2:-3}; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 NAVGPU_KNN_STATS=1 NAVGPU_KNN_MODE=${MODE:-1}
for r in $(seq $ROUNDS); do
  for lib in ${VDIR:-nav-slam_amd/lib/variants}/*.so; do
    case $lib in *stamps*|*check*) continue;; esac
    timeout -k 10 120 python3 scripts/knn_probe.py --occ 5 --reps 20 --lib $lib > "$OUT/p.json" 2>&1 || { cat "$OUT/p.json"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/p.json').read().strip().splitlines()[-1]); print('$(basename $lib)', round(d['query_us'],1), round(d['build_us'],1), d['slow_lanes'])"
  done
done
