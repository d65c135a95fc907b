#!/bin/bash
# r5: k-NN GPU tests, then the query pass A/B (NAVGPU_KNN_MODE 1 = k_knnw,
# 2 = k_knng) isolated (knn_probe.py) and in the two-in-flight bench step.
#   scripts/r5_knng_ab.sh OUTTAG [pytest -k expr]
OUT=gpurun_out/$1; mkdir -p "$OUT"; KEXPR=${2:-knn}
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
if [ "$KEXPR" != "none" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
    --timeout-method thread -k "$KEXPR" > "$OUT/pytest.log" 2>&1; rc=$?
  tail -n 3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2; do
  for m in 1 2; do
    NAVGPU_KNN_STATS=1 NAVGPU_KNN_MODE=$m timeout -k 10 120 python3 scripts/knn_probe.py --reps 20 \
      > "$OUT/probe_m${m}_r$r.json" 2> "$OUT/probe_m${m}_r$r.err" || { tail -5 "$OUT/probe_m${m}_r$r.err"; exit 1; }
    echo "mode $m: $(cat "$OUT/probe_m${m}_r$r.json")"
  done
done
BENCH_ARGS="" bash scripts/env_ab.sh "$1/ab" 2 "NAVGPU_KNN_MODE=1" "NAVGPU_KNN_MODE=2"
