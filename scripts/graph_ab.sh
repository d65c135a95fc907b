#!/bin/bash
O=gpurun_out/graph; mkdir -p $O
for r in 1 2; do
for a in "--inflight 1" "--inflight 1 --graph" "--inflight 2"; do
  timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-stream-copy $a --json-out $O/b.json > $O/b.log 2>&1 || { tail $O/b.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('$a'.ljust(24), d['ms_per_step'], d['kernel_us'])"
done; done
