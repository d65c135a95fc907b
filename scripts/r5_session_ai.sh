#!/bin/bash
# k_knng LDS image size (records per round) under 3 pairs in flight
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 3 "NAVGPU_AB_ARM=rec800" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_rec640.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_rec704.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_rec960.so"
