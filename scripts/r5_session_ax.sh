#!/bin/bash
# k_bbox_partial with clamped unconditional loads (U=4 default, U=8) vs HEAD: kernel trace + k-NN tests
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "knn" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for r in 1 2; do
for v in clamp4 head; do
  L=""; [ $v = head ] && L="nav-slam_amd/lib/variants/libnavgpu_bbhead.so"; [ $v = u8 ] && L="nav-slam_amd/lib/variants/libnavgpu_bbu8.so"
  NAVGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr_${v}_$r" -o run --output-format csv -- python3 scripts/knn_probe.py --reps 10 > "$OUT/tr_$v.log" 2>&1 || { tail "$OUT/tr_$v.log"; exit 1; }
  python3 -c "
import csv,re
for r in csv.DictReader(open('$OUT/tr_${v}_$r/run_kernel_stats.csv')):
    m=re.search(r'k_\w+',r['Name'])
    if m and m.group(0) in ('k_bin_fine','k_bin_hist','k_bin_scatter','k_bbox_partial'): print('$v', m.group(0), round(float(r['AverageNs'])/1e3,2))"
done
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 3 "NAVGPU_AB_ARM=clamp" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_bbhead.so"
