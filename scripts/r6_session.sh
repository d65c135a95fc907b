export NAVSLAM_QUIET=1; OUT=gpurun_out/r6k; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "k5_" > $OUT/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "PASSED|FAILED|Error|assert" $OUT/pytest.log | head -20; [ $rc -ne 0 ] && exit $rc
NAVSLAM_HOST_TREES=0 timeout -k 10 400 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-traffic-json --json-out $OUT/bench_k5_fast_lazy.json > $OUT/bench_k5.log 2>&1; echo bench rc=$?
python3 -c "import json; d=json.load(open('$OUT/bench_k5_fast_lazy.json')); print(d['ms_per_step'], d['pose_vs_trace'], d['cpu_baseline'] and d['cpu_baseline'].get('pose_rmse_mm'))"
