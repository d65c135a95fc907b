#!/bin/bash
# hardware queues per process (GPU_MAX_HW_QUEUES, default 4) x pairs in flight
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in "4 3" "8 3" "16 3" "8 4" "8 2"; do
    set -- $v
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 120 python3 bench.py --inflight $2 --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -20 "$OUT/b.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('queues $1 inflight $2', d['ms_per_step'], round(d['value']/1e9, 3))"
  done
done
