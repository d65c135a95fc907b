#!/bin/bash
# quick session: GPU parity tests (optionally filtered) + k-NN probe sweep
TAG=${1:-q}; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
PYTHONUNBUFFERED=1 timeout -k 10 900 python3 -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread "$@" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 4 "$OUT/pytest.log"
if fatal $rc; then exit $rc; fi
for occ in ${OCCS:-5}; do
  NAVGPU_KNN_OCC=$occ timeout -k 10 300 python3 scripts/knn_probe.py --occ $occ >> "$OUT/probe.log" 2>&1; rc=$?
  echo "probe occ=$occ rc=$rc"; if fatal $rc; then exit $rc; fi
done
grep occ "$OUT/probe.log"
