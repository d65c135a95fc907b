#!/bin/bash
# Build experimental libnavgpu variants (compile-time knobs / timing-only
# ablations) into nav-slam_amd/lib/variants/ for knn_probe.py --lib.
cd "$(dirname "$0")/.." || exit 1
rm -rf nav-slam_amd/lib/variants; mkdir -p nav-slam_amd/lib/variants
build() {  # build <name> <defines...>
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC \
    -Iinclude "$@" -shared -o "nav-slam_amd/lib/variants/libnavgpu_$name.so" \
    nav-slam_amd/csrc/navgpu.hip &
}
build r2048 -DNAVGPU_TILE_REC=2048 -DNAVGPU_TILE_QUERIES=220.0
build t192 -DNAVGPU_TILE_THREADS=192 -DNAVGPU_TILE_REC=2048 -DNAVGPU_TILE_QUERIES=165.0
build t128 -DNAVGPU_TILE_THREADS=128 -DNAVGPU_TILE_REC=1536 -DNAVGPU_TILE_QUERIES=110.0
build t320 -DNAVGPU_TILE_THREADS=320 -DNAVGPU_TILE_REC=3072 -DNAVGPU_TILE_QUERIES=300.0
build t192r16 -DNAVGPU_TILE_THREADS=192 -DNAVGPU_TILE_REC=1600 -DNAVGPU_TILE_QUERIES=165.0
wait
ls nav-slam_amd/lib/variants
