#!/bin/bash
# k_knn_slow grid size (2048 / 1024 / 512 workgroups): trace + bench A/B
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in sb2048 sb1024 sb512; do
  L=""; [ $v != sb2048 ] && L="nav-slam_amd/lib/variants/libnavgpu_$v.so"
  NAVGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$v" -o run --output-format csv -- python3 scripts/knn_probe.py --reps 10 > "$OUT/tr_$v.log" 2>&1 || { tail "$OUT/tr_$v.log"; exit 1; }
  python3 -c "
import csv,re
for r in csv.DictReader(open('$OUT/tr_$v/run_kernel_stats.csv')):
    m=re.search(r'k_\w+',r['Name'])
    if m and m.group(0) in ('k_knn_slow','k_knng'): print('$v', m.group(0), round(float(r['AverageNs'])/1e3,2))"
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 3 "NAVGPU_AB_ARM=sb2048" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_sb1024.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_sb512.so"
