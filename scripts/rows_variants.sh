#!/bin/bash
# per-row screen timing (scripts/rows_screen_probe.py, default knobs only) per library variant
OUT=gpurun_out/${1:-rv}; mkdir -p "$OUT"
for lib in "" nav-slam_amd/lib/variants/*.so; do
  n=$(basename "${lib:-base}" .so)
  timeout -k 10 200 python3 scripts/rows_screen_probe.py --default-only ${lib:+--lib $lib} > "$OUT/$n.log" 2>&1; rc=$?
  echo "$n rc=$rc"; grep "S=None NT=None" "$OUT/$n.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
