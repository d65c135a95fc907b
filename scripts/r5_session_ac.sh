#!/bin/bash
# K3 pairs in flight x curvature stream (NAVGPU_PAIR_SIDE), two interleaved rounds
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in "2 1" "2 0" "3 0" "4 0" "3 1"; do
    set -- $v
    NAVGPU_PAIR_SIDE=$2 timeout -k 10 120 python3 bench.py --inflight $1 --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -20 "$OUT/b.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('inflight $1 side $2', d['ms_per_step'], round(d['value']/1e9, 3))"
  done
done
