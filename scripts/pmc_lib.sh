#!/bin/bash
# SQ counter pass over knn_probe with a given library (LIB=...), one --pmc run
TAG=${1:-pl}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp NAVSLAM_QUIET=1
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS} -d "$OUT/pmc" -o run --output-format csv -- python3 scripts/knn_probe.py --occ 5 --reps 2 ${LIB:+--lib $LIB} > "$OUT/pmc.log" 2>&1; rc=$?
echo "pmc rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python3 scripts/pmc_summary.py "$OUT" | grep -A1 "k_knn<8, false" | cut -c1-400
