#!/bin/bash
# Per-kernel durations of the K3 step in the bench's own regime (9 resident
# pairs rotated, so the build reads its inputs from HBM, one pair at a time):
# r6_trace_cold.sh TAG label:lib.so ...   (empty lib = the in-tree build)
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp NAVSLAM_QUIET=1
for spec in "$@"; do
  label=${spec%%:*}; lib=${spec#*:}
  NAVGPU_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$label" -o run --output-format csv -- python3 bench.py --inflight 1 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic-json --no-stream-copy --json-out "$OUT/$label.json" > "$OUT/$label.log" 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$label rc=$rc"; tail -3 "$OUT/$label.log"; exit $rc; fi
  python3 scripts/kstats.py "$label" "$(find "$OUT/$label" -name '*kernel_stats.csv' | head -1)"
done
