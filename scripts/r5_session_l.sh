#!/bin/bash
# k_knng timing-only ablations: isolated query time and FETCH per variant
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 TMPDIR=/tmp NAVGPU_KNN_MODE=2
V=nav-slam_amd/lib/variants
for r in 1 2; do
for v in "" a1 a2 a4 a8 a15; do
  l=${v:+$V/libnavgpu_$v.so}
  timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 ${l:+--lib $l} > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
  echo "probe ${v:-base}: $(python3 -c "import json; d=json.load(open('$OUT/probe.json')); print(round(d['query_us'],1), round(d['build_us'],1))")"
done
done
for v in a1 a2 a8; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_$v" -o run --output-format csv -- python3 scripts/knn_probe.py --reps 2 --lib $V/libnavgpu_$v.so > "$OUT/pmc_$v.log" 2>&1 || exit 1
done
python3 scripts/pmc_summary.py "$OUT"
