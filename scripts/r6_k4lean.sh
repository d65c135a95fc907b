#!/bin/bash
# r6: the lean tie kernel's threads per row (NAVGPU_LEAN_NT; profiles/r6/k4i_lean_threads_ab.txt):
# the per-row GPU tests at the default (512), then K4 integer-mm and f64 lines at 256 / 512
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "rows or lean or batch or kd_build or nth_element" > gpurun_out/lean_tests.log 2>&1; rc=$?; tail -2 gpurun_out/lean_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for nt in 256 512; do for im in "--integer-mm" ""; do
  NAVGPU_LEAN_NT=$nt timeout -k 10 300 python3 bench.py --workload k4 $im --steps 10 --warmup 2 --no-cpu-baseline --no-stream-copy > gpurun_out/lean_$nt.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/lean_$nt.json').read().strip().splitlines()[-1]); print('k4${im:+i} nt$nt', d['ms_per_step'], d['value'])"
done; done; done
