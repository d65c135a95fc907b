#!/bin/bash
# r4: k_bin_hist grid parameters by value (A/B build_us), knn tests
TAG=${1:-r4s18}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "knn or pair or smoke" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
VDIR=nav-slam_amd/lib/variants_h bash scripts/r4_var.sh "$TAG/h" 3
