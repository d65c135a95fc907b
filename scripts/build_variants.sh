#!/bin/bash
# Build experimental libnavgpu variants (compile-time tile knobs) into
# nav-slam_amd/lib/variants/ for side-by-side timing with knn_probe.py --lib.
cd "$(dirname "$0")/.." || exit 1
mkdir -p nav-slam_amd/lib/variants
build() {  # build <name> <defines...>
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC \
    -Iinclude "$@" -shared -o "nav-slam_amd/lib/variants/libnavgpu_$name.so" \
    nav-slam_amd/csrc/navgpu.hip &
}
build t256_r2048_q220 -DNAVGPU_TILE_THREADS=256 -DNAVGPU_TILE_REC=2048 -DNAVGPU_TILE_QUERIES=220.0
build t256_r2048_q250 -DNAVGPU_TILE_THREADS=256 -DNAVGPU_TILE_REC=2048 -DNAVGPU_TILE_QUERIES=250.0
build t512_r4096_q440 -DNAVGPU_TILE_THREADS=512 -DNAVGPU_TILE_REC=4096 -DNAVGPU_TILE_QUERIES=440.0
build t512_r6144_q480 -DNAVGPU_TILE_THREADS=512 -DNAVGPU_TILE_REC=6144 -DNAVGPU_TILE_QUERIES=480.0
build t128_r1536_q120 -DNAVGPU_TILE_THREADS=128 -DNAVGPU_TILE_REC=1536 -DNAVGPU_TILE_QUERIES=120.0
wait
ls -la nav-slam_amd/lib/variants
