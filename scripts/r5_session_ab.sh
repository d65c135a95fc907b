#!/bin/bash
# staged map-slot download, one DMA + chunked parallel copy-out: tests, K5 A/B
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1 NAVSLAM_HOST_TREES=0
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "copy_paths or download_staged" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for rep in 1 2; do
for v in "NAVSLAM_D2H=0" "NAVSLAM_D2H=0 NAVGPU_COPY_THREADS=7" "NAVSLAM_D2H=0 NAVGPU_STAGE_PIECE_KB=2048" "NAVSLAM_D2H=2"; do
env $v timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-cpu-baseline --json-out "$OUT/k5.json" > "$OUT/k5.log" 2>&1 || { tail "$OUT/k5.log"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/k5.json')); print('$v rep=$rep', d['ms_per_step'], d['copy_floor_ms'], d['frac_of_copy_floor'])"
done
done
