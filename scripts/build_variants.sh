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
build base
build f512s9 -DNAVGPU_BIN_FINE_THREADS=512 -DNAVGPU_BIN_MIN_SHIFT=9
build f256s8 -DNAVGPU_BIN_FINE_THREADS=256 -DNAVGPU_BIN_MIN_SHIFT=8
build f512s10 -DNAVGPU_BIN_FINE_THREADS=512 -DNAVGPU_BIN_MIN_SHIFT=10
build f256s9 -DNAVGPU_BIN_FINE_THREADS=256 -DNAVGPU_BIN_MIN_SHIFT=9
wait
ls nav-slam_amd/lib/variants
