#!/bin/bash
# k_knng chunks-per-wave variants, isolated probe (mode 2), two rounds
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for r in 1 2; do
for v in default cpw2 cpw2b cpw3b; do
  LIBARG=""; [ $v != default ] && LIBARG="--lib nav-slam_amd/lib/variants/libnavgpu_$v.so"
  NAVGPU_KNN_STATS=1 NAVGPU_KNN_MODE=2 timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 $LIBARG \
    > "$OUT/probe_${v}_r$r.json" 2> "$OUT/probe_${v}_r$r.err" || { tail -5 "$OUT/probe_${v}_r$r.err"; exit 1; }
  echo "$v: $(cat "$OUT/probe_${v}_r$r.json")"
done
done
