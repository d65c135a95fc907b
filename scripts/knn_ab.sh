#!/bin/bash
# k-NN A/B session: the k-NN GPU parity tests, then knn_probe on the in-tree
# library and on every variant under nav-slam_amd/lib/variants
TAG=${1:-ab}; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 NAVGPU_KNN_STATS=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
PYTHONUNBUFFERED=1 timeout -k 10 600 python3 -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 4 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then exit $rc; fi
for lib in "" nav-slam_amd/lib/variants/*.so; do
  timeout -k 10 120 python3 scripts/knn_probe.py --occ ${OCC:-5} --reps 20 ${lib:+--lib $lib} >> "$OUT/probe.log" 2>&1; rc=$?
  echo "probe $lib rc=$rc"; if fatal $rc; then exit $rc; fi
done
cat "$OUT/probe.log"
