#!/bin/bash
# r4: staged target placement A/B (build_us), then evidence part 2 (PMC of
# the per-row workloads)
TAG=${1:-r4s15}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
VDIR=nav-slam_amd/lib/variants bash scripts/r4_var.sh "$TAG/ts" 3 || exit $?
PARTS="pmc" SKIP_TESTS=1 bash scripts/round_evidence.sh r4e2
