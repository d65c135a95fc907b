#!/bin/bash
# full GPU tests at the k_knng default, the K5 map-call probe, a K5 copy trace
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 120 python3 scripts/k5_map_probe.py > "$OUT/map_probe.json" 2> "$OUT/map_probe.err" || { tail "$OUT/map_probe.err"; exit 1; }
python3 -c "import json; [print(k, v) for k, v in json.load(open('$OUT/map_probe.json')).items()]"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
NAVSLAM_HOST_TREES=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/prof" -o k5 -- python3 bench.py --workload k5 --k5-mode fast --steps 30 --warmup 5 --no-cpu-baseline --json-out "$OUT/k5_prof.json" > "$OUT/k5_prof.log" 2>&1 || { tail "$OUT/k5_prof.log"; exit 1; }
python3 scripts/k5_timeline.py "$OUT/prof"
