#!/bin/bash
# SQ counter passes over the K2 per-row bench (k_rows_screen), one --pmc pass per group
OUT=gpurun_out/${1:-sq_k4}; mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 bench.py --workload k4 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic-json --no-stream-copy > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run pmc_a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS
run pmc_b SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_rows_screen" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc): print(f"{k:28s} {acc[k] / max(n[k], 1):.4g} per dispatch ({n[k]} rows)")
PY
