#!/bin/bash
# r3: K3 bench lines A/B over variant libraries (NAVGPU_LIB), interleaved
TAG=${1:-bab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
for r in $(seq ${ROUNDS:-2}); do
  for v in base ${VARIANTS}; do
    lib=""; [ "$v" != base ] && lib="$PWD/nav-slam_amd/lib/variants/libnavgpu_$v.so"
    NAVGPU_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-stream-copy ${ARGS:---steps 40} > "$OUT/$v.$r.json" 2>/dev/null || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys;d=json.load(open('$OUT/$v.$r.json'));print('$v', d['ms_per_step'], json.dumps(d['kernel_us']), json.dumps(d['kernel_us_isolated']))"
  done
done
