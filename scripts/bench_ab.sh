#!/bin/bash
# K3 bench.py A/B over the variant builds in nav-slam_amd/lib/variants
# (NAVGPU_LIB), interleaved rounds on one box; prints ms_per_step per build.
# VDIR = the variant directory, BENCH_ARGS = extra bench.py arguments
# (e.g. "--workload k2 --integer-mm").
OUT=gpurun_out/${1:-bench_ab}; ROUNDS=${2:-3}; mkdir -p "$OUT"
export NAVSLAM_QUIET=1
for r in $(seq "$ROUNDS"); do
  for l in ${VDIR:-nav-slam_amd/lib/variants}/*.so; do
    NAVGPU_LIB=$l timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline $BENCH_ARGS \
      --no-stream-copy --json-out "$OUT/b.json" > /dev/null 2>&1 || exit 1
    python3 - "$l" "$OUT/b.json" <<'PY'
import json, os, sys
d = json.load(open(sys.argv[2]))
print(os.path.basename(sys.argv[1]), d["ms_per_step"], d.get("kernel_us_isolated"))
PY
  done
done
