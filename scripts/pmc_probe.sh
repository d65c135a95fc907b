#!/bin/bash
# PMC passes over the K3 k-NN probe (isolated pair): FETCH_SIZE, WRITE_SIZE,
# L2 hits/misses; one --pmc pass each, no trace domains.
#   [NAVGPU_KNN_MODE=m] scripts/pmc_probe.sh OUTTAG
OUT=gpurun_out/${1:-pmcp}; mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 scripts/knn_probe.py --reps 2 > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run pmc_fetch FETCH_SIZE
run pmc_write WRITE_SIZE
run pmc_tcc TCC_HIT_sum TCC_MISS_sum
python3 scripts/pmc_summary.py "$OUT" all
