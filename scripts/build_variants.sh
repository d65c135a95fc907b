#!/bin/bash
# Build experimental libnavgpu variants (compile-time tile knobs) into
# nav-slam_amd/lib/variants/ for side-by-side timing with knn_probe.py --lib.
cd "$(dirname "$0")/.." || exit 1
rm -rf nav-slam_amd/lib/variants; mkdir -p nav-slam_amd/lib/variants
build() {  # build <name> <defines...>
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC \
    -Iinclude "$@" -shared -o "nav-slam_amd/lib/variants/libnavgpu_$name.so" \
    nav-slam_amd/csrc/navgpu.hip &
}
build base -DNAVGPU_TILE_THREADS=256 -DNAVGPU_TILE_REC=2048
build r1024_w5 -DNAVGPU_TILE_THREADS=256 -DNAVGPU_TILE_REC=1024 -DNAVGPU_TILE_QUERIES=110.0 -DNAVGPU_KNN_MINW=5
build r1024_w6 -DNAVGPU_TILE_THREADS=256 -DNAVGPU_TILE_REC=1024 -DNAVGPU_TILE_QUERIES=110.0 -DNAVGPU_KNN_MINW=6
build r768_w8 -DNAVGPU_TILE_THREADS=256 -DNAVGPU_TILE_REC=768 -DNAVGPU_TILE_QUERIES=80.0 -DNAVGPU_KNN_MINW=8
build t128_r1024_w6 -DNAVGPU_TILE_THREADS=128 -DNAVGPU_TILE_REC=1024 -DNAVGPU_TILE_QUERIES=110.0 -DNAVGPU_KNN_MINW=6
wait
ls nav-slam_amd/lib/variants
