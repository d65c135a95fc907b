#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
timeout -k 10 300 python3 bench.py --json-out "$OUT/k3.json" > "$OUT/k3.log" 2>&1 || { tail -20 "$OUT/k3.log"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/k3.json')); r=d['roofline']
print(d['ms_per_step'], round(d['value']/1e9,3), r['avg_us'], r['frac'], r.get('avg_us_isolated'), r['build'], d['kernel_us'], d['kernel_us_isolated'], r['trace'])"
NAVSLAM_HOST_TREES=0 timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-cpu-baseline --json-out "$OUT/k5.json" > "$OUT/k5.log" 2>&1 || { tail "$OUT/k5.log"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/k5.json')); print(d['ms_per_step'], d['frac_of_copy_floor'], d['kernel_us'], d['roofline'])"
