#!/bin/bash
# r5 session c: kernel traces (isolated probe and two-in-flight bench) of
# k_knng, the occupancy knob under k_knng, bench A/B against k_knnw
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 TMPDIR=/tmp
for occ in 5 4.5 4 3.5; do
  NAVGPU_KNN_STATS=1 NAVGPU_KNN_OCC=$occ timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 \
    > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
  echo "occ $occ: $(cat "$OUT/probe.json")"
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/tr_iso" -o run --output-format csv -- \
  python3 scripts/knn_probe.py --reps 10 > "$OUT/tr_iso.log" 2>&1 || { tail "$OUT/tr_iso.log"; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/tr_bench" -o run --output-format csv -- \
  python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-stream-copy --json-out "$OUT/tr_bench.json" \
  > "$OUT/tr_bench.log" 2>&1 || { tail "$OUT/tr_bench.log"; exit 1; }
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_KNN_MODE=1" "NAVGPU_KNN_MODE=2" "NAVGPU_KNN_MODE=2 NAVGPU_KNN_OCC=4"
