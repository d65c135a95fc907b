#!/bin/bash
# K5 copy paths: parity test, then an A/B of NAVSLAM_D2H x NAVGPU_D2H_PIECE_KB (300 frames each, twice)
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 NAVSLAM_HOST_TREES=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "copy_paths" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for rep in 1 2; do
for v in 0,4096 1,4096 0,0 1,0; do
d=${v%,*}; p=${v#*,}
NAVSLAM_D2H=$d NAVGPU_D2H_PIECE_KB=$p timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-cpu-baseline --json-out "$OUT/k5_d${d}_p${p}_$rep.json" > "$OUT/k5_d${d}_p${p}_$rep.log" 2>&1 || { tail "$OUT/k5_d${d}_p${p}_$rep.log"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/k5_d${d}_p${p}_$rep.json')); print('side=$d piece=$p rep=$rep', d['ms_per_step'], d['copy_floor_ms'], d['frac_of_copy_floor'])"
done
done
