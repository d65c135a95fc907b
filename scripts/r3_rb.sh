#!/bin/bash
# r3: k_rows_build A/B over the variant libraries (interleaved rounds)
TAG=${1:-rb}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in default ${VARIANTS:-nopre stamps stampsnopre}; do
    lib=""; [ "$v" != default ] && lib="--lib nav-slam_amd/lib/variants/libnavgpu_$v.so"
    timeout -k 10 120 python3 scripts/rows_build_probe.py $lib --tag "$v" >> "$OUT/probe.jsonl" 2>> "$OUT/probe.err" || { echo "FAIL $v"; exit 1; }
  done
done
cat "$OUT/probe.jsonl"
