#!/bin/bash
# K5 copies: the copy probe, then the K5 loop under a kernel + copy trace
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python3 scripts/copy_probe.py > "$OUT/copy_probe.json" 2> "$OUT/copy_probe.err" || { tail "$OUT/copy_probe.err"; exit 1; }
cat "$OUT/copy_probe.json"
NAVSLAM_HOST_TREES=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/prof" -o k5 -- python3 bench.py --workload k5 --k5-mode fast --steps 30 --warmup 5 --no-cpu-baseline --json-out "$OUT/k5_prof.json" > "$OUT/k5_prof.log" 2>&1 || { tail "$OUT/k5_prof.log"; exit 1; }
find "$OUT/prof" -name "*.csv" | head -20
