#!/bin/bash
# r3 k-NN sweep: settings on the product build, then phase stamps and ablations
TAG=${1:-s}; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
V=nav-slam_amd/lib/variants
run() { echo "== $*" >> "$OUT/sweep.log"; timeout -k 10 300 python3 scripts/knn_sweep.py "$@" >> "$OUT/sweep.log" 2>&1; rc=$?; echo "rc=$rc"; if fatal $rc; then exit $rc; fi; }
run ${CONFIGS:-"SX=4" "SX=2" "SX=1" "SX=4,LAMBDA=16" "SX=4,LAMBDA=30"}
for v in ${VARIANTS:-stamps noquery noexact}; do run --lib $V/libnavgpu_$v.so "SX=4"; done
grep -v amdgpu.ids "$OUT/sweep.log"
