#!/bin/bash
# kernel trace + PMC passes (one --pmc pass per argument) of an arbitrary
# python script: scripts/prof_cmd.sh <tag> <script.py> [pmc-set ...]
OUT=gpurun_out/${1:-prof}; SCRIPT=$2; shift 2; mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 $SCRIPT > "$OUT/trace.log" 2>&1; rc=$?; echo "trace rc=$rc"; fatal $rc && exit $rc
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d "$OUT/pmc$i" -o run --output-format csv -- python3 $SCRIPT > "$OUT/pmc$i.log" 2>&1; rc=$?; echo "pmc$i rc=$rc"; fatal $rc && exit $rc
done
echo done
