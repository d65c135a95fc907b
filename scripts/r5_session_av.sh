#!/bin/bash
# wave-group Lomuto levels in the per-row tree build: tree tests first (each
# GPU step under its own limit), then K2i / K4i / K5-host-trees A/B
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "kd_build or rows_match_k2 or rows_match_batch" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
grep -c PASSED "$OUT/pytest.log"; tail -1 "$OUT/pytest.log"
for r in 1 2; do
  for v in "NAVGPU_AB_ARM=group128" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_nogroup.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_nosleep.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_nosleep256.so"; do
    env $v timeout -k 10 120 python3 bench.py --workload k2 --integer-mm --steps 10 --no-cpu-baseline --no-stream-copy --json-out "$OUT/k2i.json" > "$OUT/k2i.log" 2>&1 || { tail -20 "$OUT/k2i.log"; exit 1; }
    env $v timeout -k 10 200 python3 bench.py --workload k4 --integer-mm --steps 3 --warmup 1 --no-cpu-baseline --no-stream-copy --json-out "$OUT/k4i.json" > "$OUT/k4i.log" 2>&1 || { tail -20 "$OUT/k4i.log"; exit 1; }
    python3 -c "import json; a=json.load(open('$OUT/k2i.json')); b=json.load(open('$OUT/k4i.json')); print('$v'[-28:], 'k2i', a['ms_per_step'], 'k4i', b['ms_per_step'])"
  done
done
