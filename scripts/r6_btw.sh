#!/bin/bash
# r6 one-off (profiles/r6/k2i_chain_ab.txt, threshold sweep): build the variants first with
#   scripts/build_variants.sh st_base:"-DNAVGPU_STAMPS" st_btw1024:"-DNAVGPU_STAMPS -DNAVGPU_BLOCK_TO_WAVE=1024" \
#     st_btw8192:"-DNAVGPU_STAMPS -DNAVGPU_BLOCK_TO_WAVE=8192" btw512:"-DNAVGPU_BLOCK_TO_WAVE=512" \
#     btw1024:"-DNAVGPU_BLOCK_TO_WAVE=1024" btw8192:"-DNAVGPU_BLOCK_TO_WAVE=8192"
for v in st_base st_btw1024 st_btw8192; do timeout -k 10 120 python3 scripts/rows_probe.py --integer --lib nav-slam_amd/lib/variants/libnavgpu_$v.so || exit 1; done
SKIP_TESTS=1 WORKLOADS="k2 k4" bash scripts/r6_tie.sh r6t10 2 btw512 btw1024 btw8192
