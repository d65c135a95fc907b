#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/k2t; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 bench.py --workload k2 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic-json --no-stream-copy > $O/log 2>&1 || exit 1
cut -d, -f1-5 $O/t/run_kernel_stats.csv | sed 's/(anonymous namespace):://g' | cut -c1-150
