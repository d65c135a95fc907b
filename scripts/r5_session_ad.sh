#!/bin/bash
# coalesced k_nb_fill list writes: k-NN + copy-path tests, build time A/B
# (NAVGPU_NB_SPAN=0 = run-by-run writes), bench A/B, K5 with host trees
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "knn or copy_paths" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for sp in "" 0; do
    NAVGPU_NB_SPAN=$sp timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 > "$OUT/probe.json" 2> "$OUT/probe.err" || { tail -5 "$OUT/probe.err"; exit 1; }
    echo "span=${sp:-default}: $(cat "$OUT/probe.json")"
  done
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_NB_SPAN=" "NAVGPU_NB_SPAN=0"
timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 100 --warmup 5 --no-cpu-baseline --json-out "$OUT/k5_trees.json" > "$OUT/k5_trees.log" 2>&1 || { tail "$OUT/k5_trees.log"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/k5_trees.json')); print('k5 host trees', d['ms_per_step'], d['frac_of_copy_floor'])"
