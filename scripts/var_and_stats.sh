#!/bin/bash
# variant probe (every lib under nav-slam_amd/lib/variants) + a kernel-stats
# trace of the default library on the K3 probe
OUT=gpurun_out/${1:-vs}; mkdir -p "$OUT"
export TMPDIR=/tmp
bash scripts/variants_probe.sh "${1:-vs}" || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 scripts/knn_probe.py --occ 5 --reps 10 > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py "$OUT"
