#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
  --timeout-method thread -k "lazy or twice or l9_stream or l5_stream" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest: $(tail -n 1 "$OUT/pytest.log")"; exit $rc
