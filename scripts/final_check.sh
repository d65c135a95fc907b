#!/bin/bash
# Final check: the whole GPU suite, smoke, the default bench line
TAG=${1:-final}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -n 2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -n 1 "$OUT/smoke.log"
timeout -k 10 400 python3 bench.py --json-out "$OUT/bench_k3.json" > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_k3.json')); r=d['roofline']; print('k3', d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), d['kernel_us_isolated'], d['cpu_baseline']['value'])"
