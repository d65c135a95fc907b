#!/bin/bash
# Build experimental libnavgpu variants (compile-time knobs, phase stamps,
# timing-only ablations) into nav-slam_amd/lib/variants/ for
# knn_probe.py --lib / knn_sweep.py.
# usage: [VDIR=dir] scripts/build_variants.sh [name:"-DFLAG -DFLAG2" ...]  (default: stamps)
cd "$(dirname "$0")/.." || exit 1
VDIR=${VDIR:-nav-slam_amd/lib/variants}
rm -rf "$VDIR"; mkdir -p "$VDIR"
build() {  # build <name> <defines...>
  local name=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC \
    -Iinclude "$@" -shared -o "$VDIR/libnavgpu_$name.so" \
    nav-slam_amd/csrc/navgpu.hip nav-slam_amd/csrc/knn.hip &
}
if [ $# -gt 0 ]; then
  for spec in "$@"; do build "${spec%%:*}" ${spec#*:}; done
else
  build stamps -DNAVGPU_STAMPS
fi
wait
ls "$VDIR"
