#!/bin/bash
# K2 and K4 bench lines (with the reference CPU baseline on one pair)
OUT=gpurun_out/${1:-k24}; mkdir -p "$OUT"
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python3 bench.py --workload k2 --steps 10 --json-out "$OUT/bench_k2.json" > "$OUT/k2.log" 2>&1; rc=$?; echo "k2 rc=$rc"; fatal $rc && exit $rc
timeout -k 10 400 python3 bench.py --workload k4 --steps 3 --warmup 1 --json-out "$OUT/bench_k4.json" > "$OUT/k4.log" 2>&1; rc=$?; echo "k4 rc=$rc"; fatal $rc && exit $rc
python3 - "$OUT" <<'PY'
import json, sys
for w in ("k2", "k4"):
    d = json.load(open(f"{sys.argv[1]}/bench_{w}.json"))
    r, c = d["roofline"], d["cpu_baseline"] or {}
    print(w, d["value"], d["ms_per_step"], r.get("achieved"), r.get("frac"), c.get("value"), c.get("seconds_per_pair"))
PY
