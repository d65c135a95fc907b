#!/bin/bash
# staged map-slot download: tests, K5 A/B (NAVSLAM_D2H 0 staged / 2 main / 1 side), trace
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 NAVSLAM_HOST_TREES=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "copy_paths or download_staged or l9_stream or localise_twice" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for rep in 1 2; do
for d in 0 2 1; do
NAVSLAM_D2H=$d timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-cpu-baseline --json-out "$OUT/k5_d${d}_$rep.json" > "$OUT/k5_d${d}_$rep.log" 2>&1 || { tail "$OUT/k5_d${d}_$rep.log"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/k5_d${d}_$rep.json')); print('d2h=$d rep=$rep', d['ms_per_step'], d['copy_floor_ms'], d['frac_of_copy_floor'])"
done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/prof" -o k5 -- python3 bench.py --workload k5 --k5-mode fast --steps 30 --warmup 5 --no-cpu-baseline --json-out "$OUT/k5_prof.json" > "$OUT/k5_prof.log" 2>&1 || { tail "$OUT/k5_prof.log"; exit 1; }
python3 scripts/k5_timeline.py "$OUT/prof"
