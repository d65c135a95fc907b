#!/bin/bash
# multi-segment k_curvature waves: curvature tests, then bench A/B over segments per wave
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "curvature or rows_match or rows_screen or pipelined or shim_l5" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 3 "NAVGPU_AB_ARM=curv4" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_curv1.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_curv2.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_curv8.so"
