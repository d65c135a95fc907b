#!/bin/bash
# k_knng staging from packed 12-B records vs the 16-B SRec: k-NN tests, probe, FETCH, bench A/B
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "knn" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for v in "NAVGPU_AB_ARM=pack" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_nopack.so"; do
    env $v timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
    echo "$v: $(cat "$OUT/probe.json")"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in pack nopack; do
  L=""; [ $v = nopack ] && L="nav-slam_amd/lib/variants/libnavgpu_nopack.so"
  NAVGPU_LIB=$L timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_$v" -o run --output-format csv -- python3 scripts/knn_probe.py --reps 5 > "$OUT/pmc_$v.log" 2>&1 || { tail "$OUT/pmc_$v.log"; exit 1; }
  python3 -c "
import csv,re,collections
a=collections.defaultdict(list)
for r in csv.DictReader(open('$OUT/pmc_$v/run_counter_collection.csv')):
    m=re.search(r'k_\w+',r['Kernel_Name']); a[m.group(0) if m else '?'].append(float(r['Counter_Value']))
print('$v', {k: round(sum(v)/len(v)/1024,1) for k,v in a.items() if k in ('k_knng','k_bin_fine')}, 'MB')"
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_AB_ARM=pack" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_nopack.so"
