#!/bin/bash
# sampled timing events (K3: context 0 only; K5: every 4th frame) against no
# events, and the K5 rows-query tests at 4 splits per row
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "lazy or shim or rows_query" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2 3; do
  for X in "" "--no-events"; do
    timeout -k 10 120 python3 bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy $X --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -20 "$OUT/b.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); r=d.get('roofline') or {}; print('k3', '$X' or 'sampled', d['ms_per_step'], round(d['value']/1e9, 3), r.get('avg_us'), r.get('launches'))"
    NAVSLAM_HOST_TREES=0 timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-cpu-baseline $X --json-out "$OUT/k5.json" > "$OUT/k5.log" 2>&1 || { tail "$OUT/k5.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/k5.json')); print('k5', '$X' or 'sampled', d['ms_per_step'], d['frac_of_copy_floor'], d['kernel_us'])"
  done
done
