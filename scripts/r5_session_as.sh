#!/bin/bash
# integer-mm tie pass knobs: K2i pair and K4i batch, interleaved
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in "NAVGPU_AB_ARM=default" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_blm1024.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_blm256.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_ls8.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_bnm512.so"; do
    env $v timeout -k 10 120 python3 bench.py --workload k2 --integer-mm --steps 10 --no-cpu-baseline --no-stream-copy --json-out "$OUT/k2i.json" > "$OUT/k2i.log" 2>&1 || { tail -20 "$OUT/k2i.log"; exit 1; }
    env $v timeout -k 10 200 python3 bench.py --workload k4 --integer-mm --steps 3 --warmup 1 --no-cpu-baseline --no-stream-copy --json-out "$OUT/k4i.json" > "$OUT/k4i.log" 2>&1 || { tail -20 "$OUT/k4i.log"; exit 1; }
    python3 -c "import json; a=json.load(open('$OUT/k2i.json')); b=json.load(open('$OUT/k4i.json')); print('$v'[-30:], 'k2i', a['ms_per_step'], 'k4i', b['ms_per_step'])"
  done
done
