#!/bin/bash
# K5 A/B of the shim at HEAD (variants/old) against the working tree
# built flags by k_rows_build): lazy-row tests, then 300-frame A/B against HEAD's build
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "lazy or shim or rows_query" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2 3; do
  for v in "NAVGPU_AB_ARM=new" "NAVSLAM_LIBDIR=nav-slam_amd/lib/variants/old NAVGPU_LIB=nav-slam_amd/lib/variants/old/libnavgpu.so"; do
    env $v NAVSLAM_HOST_TREES=0 timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-cpu-baseline --json-out "$OUT/k5.json" > "$OUT/k5.log" 2>&1 || { tail "$OUT/k5.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/k5.json')); print('$v'[:30], d['ms_per_step'], d['frac_of_copy_floor'], d['kernel_us'])"
  done
done
