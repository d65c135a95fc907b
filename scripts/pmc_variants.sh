#!/bin/bash
# SQ_INSTS_VALU / SQ_INSTS_LDS / SQ_WAVES of k_knn<8,false> for the in-tree library and every variant
OUT=gpurun_out/${1:-pv}; mkdir -p "$OUT"; export TMPDIR=/tmp NAVSLAM_QUIET=1
for lib in "" nav-slam_amd/lib/variants/*.so; do
  n=$(basename "${lib:-base}" .so)
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES -d "$OUT/$n" -o run --output-format csv -- python3 scripts/knn_probe.py --occ 5 --reps 2 ${lib:+--lib $lib} > "$OUT/$n.log" 2>&1; rc=$?
  if [ $rc -ne 0 ]; then echo "$n rc=$rc"; exit $rc; fi
  echo "$n $(python3 scripts/pmc_summary.py "$OUT/$n" 2>/dev/null | grep -A0 'k_knn<8, false' | grep -o "{.*}")"
done
