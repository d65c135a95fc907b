#!/bin/bash
# r6 one-off: K4 screen knobs A/B (profiles/r6/k4_screen_knobs_ab.txt); build the chunk variants first:
#   scripts/build_variants.sh ch16:"-DNAVGPU_SCREEN_CHUNK=16" ch64:"-DNAVGPU_SCREEN_CHUNK=64"
for r in 1 2; do
for spec in "base:" "nt512:NAVGPU_SCREEN_NT=512" "s2:NAVGPU_SCREEN_S=2" "ch16:NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_ch16.so" "ch64:NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_ch64.so"; do
  l=${spec%%:*}; e=${spec#*:}
  env $e timeout -k 10 300 python3 bench.py --workload k4 --steps 10 --warmup 2 --no-cpu-baseline --no-stream-copy --json-out gpurun_out/k4ab_${l}_$r.json > gpurun_out/k4ab_${l}_$r.log 2>&1 || { echo "$l failed"; tail -3 gpurun_out/k4ab_${l}_$r.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/k4ab_${l}_$r.json')); print('$l', d['ms_per_step'], d['value'])"
done; done
