#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 180 python3 scripts/k5_map_probe.py > "$OUT/map_probe.json" 2> "$OUT/map_probe.err" || { tail "$OUT/map_probe.err"; exit 1; }
python3 -c "import json; [print(k, v) for k, v in json.load(open('$OUT/map_probe.json')).items()]"
