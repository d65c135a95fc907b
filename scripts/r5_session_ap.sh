#!/bin/bash
# K3 timed region with events on the query stage only (every context) vs no events;
# the roofline span must stay a real (contended) duration
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for X in "" "--no-events"; do
    timeout -k 10 120 python3 bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy $X --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -20 "$OUT/b.log"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b.json')); r=d.get('roofline') or {}
print('k3', '$X' or 'query-events', d['ms_per_step'], round(d['value']/1e9, 3), r.get('avg_us'), r.get('launches'), r.get('avg_us_isolated'), (r.get('build') or {}).get('avg_us_isolated'), d.get('kernel_us'))"
  done
done
