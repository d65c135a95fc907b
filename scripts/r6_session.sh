export NAVSLAM_QUIET=1; OUT=gpurun_out/r6o; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -k "k5_ or shim" > $OUT/pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for p in 1 4 8; do
NAVSLAM_PIPE=$p NAVSLAM_HOST_TREES=0 timeout -k 10 300 python3 bench.py --workload k5 --k5-mode fast --steps 300 --warmup 10 --no-traffic-json --no-cpu-baseline --json-out $OUT/k5_p${p}_$r.json > $OUT/k5_p${p}_$r.log 2>&1 || exit 1
python3 -c "import json; d=json.load(open('$OUT/k5_p${p}_$r.json')); print('pipe $p', d['ms_per_step'], d['copy_floor_ms'], d['kernel_us'], d['pose_vs_trace']['rmse_mm'])"
done; done
