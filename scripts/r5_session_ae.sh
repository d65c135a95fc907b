#!/bin/bash
# k_nb_fill coalesced (default) vs run-by-run (NAVGPU_NB_SPAN=0): probe + bench A/B, and its tests
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "row_lists_both or knn_vs_brute or degenerate" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for v in "NAVGPU_AB_ARM=coalesced" "NAVGPU_NB_SPAN=0"; do
    env $v timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
    echo "$v: $(cat "$OUT/probe.json")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in coalesced runs; do
  sp=""; [ $v = runs ] && sp=0
  NAVGPU_NB_SPAN=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$v" -o run --output-format csv -- python3 scripts/knn_probe.py --reps 10 > "$OUT/tr_$v.log" 2>&1 || { tail "$OUT/tr_$v.log"; exit 1; }
  python3 -c "
import csv,re
for r in csv.DictReader(open('$OUT/tr_$v/run_kernel_stats.csv')):
    m=re.search(r'k_\w+',r['Name'])
    if m and m.group(0) in ('k_nb_fill','k_bin_fine','k_bin_scatter','k_knng'): print('$v', m.group(0), round(float(r['AverageNs'])/1e3,1))"
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_AB_ARM=coalesced" "NAVGPU_NB_SPAN=0"
