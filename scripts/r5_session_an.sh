#!/bin/bash
# K5: zero-copy fast sums (working tree vs HEAD's shim in variants/old), the
# k_rows_query_screen column splits (NAVGPU_ROWSQ_S), and K3/K5 with and
# without HIP timing events in the timed region (--no-events)
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
D=nav-slam_amd/lib/variants/old
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "lazy or shim or rows_query" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2 3; do
  for v in "NAVGPU_AB_ARM=new" "NAVSLAM_LIBDIR=$D NAVGPU_LIB=$D/libnavgpu.so" "NAVGPU_ROWSQ_S=4" "NAVGPU_ROWSQ_S=16" "NAVGPU_AB_ARM=noevents"; do
    X=""; [ "$v" = "NAVGPU_AB_ARM=noevents" ] && X="--no-events"
    env NAVSLAM_HOST_TREES=0 $v timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-cpu-baseline $X --json-out "$OUT/k5.json" > "$OUT/k5.log" 2>&1 || { tail "$OUT/k5.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/k5.json')); print('k5', '$v'[:30], d['ms_per_step'], d['frac_of_copy_floor'], d['kernel_us'])"
  done
done
for r in 1 2 3; do
  for X in "" "--no-events"; do
    timeout -k 10 120 python3 bench.py --steps 60 --warmup 6 --no-cpu-baseline --no-stream-copy $X --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -20 "$OUT/b.log"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b.json')); print('k3 events' if '$X' == '' else 'k3 no-events', d['ms_per_step'], round(d['value']/1e9, 3))"
  done
done
