#!/bin/bash
# r4: lane cutoff 16 + DPP chunk prefix in the block pass: row/kd tests,
# stamps probe, K2i / K4i lines
TAG=${1:-r4s17}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "kd or rows or lazy or shim or k1 or smoke" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 120 python3 scripts/rows_probe.py --integer --lib nav-slam_amd/lib/var_st/libnavgpu_st.so \
    > "$OUT/rp.json" 2>&1 || { tail -3 "$OUT/rp.json"; exit 1; }
  echo "st $(tail -n 1 $OUT/rp.json | cut -c1-330)"
done
for w in "k2 --integer-mm --steps 10" "k4 --integer-mm --steps 3 --warmup 1"; do
  timeout -k 10 180 python3 bench.py --workload $w --no-cpu-baseline --no-stream-copy --no-traffic-json \
    --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$w', d['value'], d['ms_per_step'])"
done
