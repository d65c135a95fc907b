#!/bin/bash
# SQ counter passes over the K3 k-NN probe (one --pmc pass per group, no trace domains)
OUT=gpurun_out/${1:-sq}; mkdir -p "$OUT"; shift
export TMPDIR=/tmp
LIBARG=${LIB:+--lib $LIB}
run() {  # run <name> counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 scripts/knn_probe.py --occ 5 --reps 2 $LIBARG > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run pmc_a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS
run pmc_b SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA
python3 scripts/pmc_summary.py "$OUT"
