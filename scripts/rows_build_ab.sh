#!/bin/bash
# Per-row build variants (lane-subtree cutoff, block levels down to 256)
# on integer-mm K2 rows (stamps builds), then K2 with 256-thread screen blocks
TAG=${1:-rows_build}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
for r in 1 2; do for l in st st_l16 st_b256 st_l16b256; do
  timeout -k 10 120 python3 scripts/rows_probe.py --integer --lib nav-slam_amd/lib/var_st/libnavgpu_$l.so \
    > "$OUT/rp.json" 2>&1 || { tail -3 "$OUT/rp.json"; exit 1; }
  echo "$l $(tail -n 1 $OUT/rp.json | cut -c1-330)"
done; done
b() {  # b <name> "<VAR=value ...>" "<bench.py arguments>"
  env $2 timeout -k 10 180 python3 bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline \
    --no-stream-copy $3 --json-out "$OUT/$1.json" > "$OUT/$1.log" 2>&1 || { tail -5 "$OUT/$1.log"; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.json')); print('$1', d['value'], d['ms_per_step'], d.get('kernel_us'))"
}
for r in 1 2; do
  b k2 "" "--workload k2" || exit 1
  b k2_nt256 "NAVGPU_SCREEN_NT=256" "--workload k2" || exit 1
  b k2_s2fuse "NAVGPU_SCREEN_S=2 NAVGPU_SCREEN_FUSE=1" "--workload k2" || exit 1
done
