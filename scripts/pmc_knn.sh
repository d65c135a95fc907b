#!/bin/bash
# PMC passes on the K3 bench (separate --pmc runs; no trace domains mixed in)
OUT=gpurun_out/${1:-pmc}; mkdir -p "$OUT"
export TMPDIR=/tmp NAVGPU_KNN_OCC=${OCC:-5}
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
echo "list rc=$?"
run() {  # run <name> counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run tcc FETCH_SIZE
run tccw WRITE_SIZE
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr
echo done
