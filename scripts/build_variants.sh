#!/bin/bash
# Build experimental libnavgpu variants (compile-time knobs / timing-only
# ablations) into nav-slam_amd/lib/variants/ for knn_probe.py --lib.
# usage: scripts/build_variants.sh [name:"-DFLAG -DFLAG2" ...]  (default: the k-NN ablation set)
cd "$(dirname "$0")/.." || exit 1
rm -rf nav-slam_amd/lib/variants; mkdir -p nav-slam_amd/lib/variants
build() {  # build <name> <defines...>
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC \
    -Iinclude "$@" -shared -o "nav-slam_amd/lib/variants/libnavgpu_$name.so" \
    nav-slam_amd/csrc/navgpu.hip &
}
if [ $# -gt 0 ]; then
  for spec in "$@"; do build "${spec%%:*}" ${spec#*:}; done
else
  build nosort -DNAVGPU_DBG_NOSORT
  build noout -DNAVGPU_DBG_NOOUT
  build nof64 -DNAVGPU_DBG_NOF64
  build noexact -DNAVGPU_DBG_NOEXACT
  build noins -DNAVGPU_DBG_NOINSERT
  build nostage -DNAVGPU_DBG_NOSTAGE
  build noquery -DNAVGPU_DBG_NOQUERY
fi
wait
ls nav-slam_amd/lib/variants
