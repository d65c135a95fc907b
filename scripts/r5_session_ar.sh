#!/bin/bash
# per-query block bounds (k_q_bounds) vs the wave's own npg lookups: k-NN tests, probe, trace, bench A/B
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "knn" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for v in "NAVGPU_AB_ARM=qb" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_nqb.so"; do
    env $v timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
    echo "$v: $(cat "$OUT/probe.json")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in qb nqb; do
  L=""; [ $v = nqb ] && L="nav-slam_amd/lib/variants/libnavgpu_nqb.so"
  NAVGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$v" -o run --output-format csv -- python3 scripts/knn_probe.py --reps 10 > "$OUT/tr_$v.log" 2>&1 || { tail "$OUT/tr_$v.log"; exit 1; }
  python3 -c "
import csv,re
for r in csv.DictReader(open('$OUT/tr_$v/run_kernel_stats.csv')):
    m=re.search(r'k_\w+',r['Name'])
    if m and m.group(0) in ('k_knng','k_q_bounds','k_nb_fill'): print('$v', m.group(0), round(float(r['AverageNs'])/1e3,1))"
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 3 "NAVGPU_AB_ARM=qb" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_nqb.so"
