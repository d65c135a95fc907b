#!/bin/bash
# r4: lazy-row query screen with start chunks: lazy / shim tests, K5 lines
TAG=${1:-r4s19}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "lazy or shim or split or rows_corr or k1" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for t in 0 1; do
  NAVSLAM_HOST_TREES=$t timeout -k 10 180 python3 bench.py --workload k5 --k5-mode fast --steps 30 --warmup 2 \
    --no-cpu-baseline --no-stream-copy --no-traffic-json --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('k5f trees=$t', d['ms_per_step'], d.get('kernel_us'))"
done; done
