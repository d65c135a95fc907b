#!/bin/bash
# k_knng chunks-per-wave variants, isolated probe (mode 2), then the bench
# A/B of them and of the lean build kernels (all NAVGPU_KNN_MODE=2)
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for r in 1 2; do
for v in default cpw2 cpw2b cpw3b nb4k; do
  LIBARG=""; [ $v != default ] && LIBARG="--lib nav-slam_amd/lib/variants/libnavgpu_$v.so"
  NAVGPU_KNN_STATS=1 NAVGPU_KNN_MODE=2 timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 $LIBARG \
    > "$OUT/probe_${v}_r$r.json" 2> "$OUT/probe_${v}_r$r.err" || { tail -5 "$OUT/probe_${v}_r$r.err"; exit 1; }
  echo "$v: $(cat "$OUT/probe_${v}_r$r.json")"
done
done
bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_KNN_MODE=2" "NAVGPU_KNN_MODE=2 NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_cpw2b.so" "NAVGPU_KNN_MODE=2 NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_lean.so" "NAVGPU_KNN_MODE=2 NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_nb4k.so" "NAVGPU_KNN_MODE=1"
