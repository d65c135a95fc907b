#!/bin/bash
# K5: map slot download on the main stream (default) against the side stream
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 NAVSLAM_HOST_TREES=0
for sd in 0 1; do
NAVSLAM_SIDE_D2H=$sd NAVSLAM_PROFILE=1 timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 60 --warmup 5 --no-cpu-baseline --json-out "$OUT/k5_sd$sd.json" > "$OUT/k5_sd$sd.log" 2>&1 || { tail "$OUT/k5_sd$sd.log"; exit 1; }
grep "navslam profile" "$OUT/k5_sd$sd.log"
python3 -c "import json; d=json.load(open('$OUT/k5_sd$sd.json')); print('side=$sd', d['ms_per_step'], d['copy_floor_ms'], d['frac_of_copy_floor'], d['kernel_us'])"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/prof" -o k5 -- python3 bench.py --workload k5 --k5-mode fast --steps 30 --warmup 5 --no-cpu-baseline --json-out "$OUT/k5_prof.json" > "$OUT/k5_prof.log" 2>&1 || { tail "$OUT/k5_prof.log"; exit 1; }
