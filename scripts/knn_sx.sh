#!/bin/bash
# k-NN x-refinement sweep: GPU k-NN parity tests at each NAVGPU_KNN_SX, then
# knn_probe timings at each
TAG=${1:-sx}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 NAVGPU_KNN_STATS=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for sx in ${SXS:-1 2 3 4}; do
  NAVGPU_KNN_SX=$sx PYTHONUNBUFFERED=1 timeout -k 10 300 python3 -m pytest tests -m gpu -x -q --timeout 240 --timeout-method=thread -k "${PYTEST_K:-knn}" > "$OUT/pytest_sx$sx.log" 2>&1; rc=$?
  echo "pytest sx=$sx rc=$rc $(tail -n 1 $OUT/pytest_sx$sx.log)"; if [ $rc -ne 0 ]; then exit $rc; fi
done
for sx in ${SXS:-1 2 3 4}; do
  NAVGPU_KNN_SX=$sx timeout -k 10 120 python3 scripts/knn_probe.py --occ ${OCC:-5} --reps 20 > "$OUT/probe_sx$sx.log" 2>&1; rc=$?
  echo "sx=$sx $(grep '^{' $OUT/probe_sx$sx.log)"; if fatal $rc; then exit $rc; fi
done
