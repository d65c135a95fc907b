#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
for p in 1 0; do
NAVSLAM_HOST_TREES=0 NAVSLAM_PROFILE=$p timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 60 --warmup 5 --no-cpu-baseline --json-out "$OUT/k5_lazy_p$p.json" > "$OUT/k5_lazy_p$p.log" 2>&1 || { tail "$OUT/k5_lazy_p$p.log"; exit 1; }
grep "navslam profile" "$OUT/k5_lazy_p$p.log"
python3 -c "import json; d=json.load(open('$OUT/k5_lazy_p$p.json')); print('profile=$p', d['ms_per_step'], d['copy_floor_ms'], d['frac_of_copy_floor'], d['kernel_us'])"
done
