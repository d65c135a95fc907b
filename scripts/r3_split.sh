#!/bin/bash
# CU-split A/B (navgpu_set_cu_split): the K3 bench under several splits, after
# the safe bit-order probe and the K3 parity tests with the split on.
set -o pipefail
O=gpurun_out/split
mkdir -p $O
timeout -k 10 60 ./bench_micro/cu_mask probe > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 3; }
timeout -k 10 120 ./bench_micro/cu_mask > $O/cu_mask.txt 2>&1 || exit 4
NAVGPU_CU_SPLIT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "knn_vs_brute or knn_hard or k3_full or pair_knn or l9_scan" \
  > $O/pytest_split4.log 2>&1 || { tail -30 $O/pytest_split4.log; exit 5; }
for sp in "" 4 6 8 4,28,0 3 2; do
  tag=${sp:-off}; tag=${tag//,/_}
  timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-stream-copy \
    ${sp:+--cu-split $sp} --json-out $O/bench_$tag.json > $O/bench_$tag.log 2>&1 || exit 6
  python - $O/bench_$tag.json "$tag" <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); r=d["roofline"]
print(sys.argv[2], "ms/step", d["ms_per_step"], "value %.3g" % d["value"], "q", r["avg_us"], "b", r["build"]["avg_us"], "curv", d["kernel_us"].get("curvature"), "iso", d["kernel_us_isolated"])
PY
done
