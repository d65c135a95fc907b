#!/bin/bash
OUT=gpurun_out/$1; mkdir -p "$OUT"
timeout -k 10 180 python3 scripts/copy_probe.py > "$OUT/copy_probe.json" 2> "$OUT/copy_probe.err" || { tail "$OUT/copy_probe.err"; exit 1; }
python3 -c "import json; [print(k, v) for k, v in json.load(open('$OUT/copy_probe.json')).items()]"
