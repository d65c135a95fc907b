#!/bin/bash
# r3 k-NN iteration: global-mode parity tests, then the isolated K3 probe.
TAG=${1:-k}; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "${TESTS:-knn}" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 5 "$OUT/pytest.log"
if fatal $rc; then exit $rc; fi
NAVGPU_KNN_STATS=1 timeout -k 10 200 python3 scripts/knn_probe.py --occ ${OCC:-5} "$@" > "$OUT/probe.log" 2>&1; rc=$?
echo "probe rc=$rc"; tail -n 2 "$OUT/probe.log"
