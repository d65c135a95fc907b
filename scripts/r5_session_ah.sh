#!/bin/bash
# pipelined K3 (build on CUs [0,N), curvature + query on [N,all)): test, then bench A/B
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "pipelined or knn_vs_brute" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for v in "3 0" "2 64" "2 96" "3 64" "2 48" "3 96"; do
    set -- $v
    timeout -k 10 120 python3 bench.py --inflight $1 --cu-split $2 --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -20 "$OUT/b.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('inflight $1 split $2', d['ms_per_step'], round(d['value']/1e9, 3), d.get('kernel_us'))"
  done
done
