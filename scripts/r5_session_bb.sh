#!/bin/bash
# fused tie pass + fast sums: tests, then K5 lazy A/B against HEAD's build (variants/old)
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
D=nav-slam_amd/lib/variants/old
#timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "lazy or shim or rows_query" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
#tail -1 "$OUT/pytest.log"
for r in 1 2 3; do
  for v in "NAVSLAM_LAZY_CORR=1" "NAVSLAM_LAZY_CORR=0"; do
    env NAVSLAM_HOST_TREES=0 $v timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-cpu-baseline --json-out "$OUT/k5.json" > "$OUT/k5.log" 2>&1 || { tail "$OUT/k5.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/k5.json')); print('$v'[:20], d['ms_per_step'], d['frac_of_copy_floor'], d['kernel_us'])"
  done
done
