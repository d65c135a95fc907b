export NAVSLAM_QUIET=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "knn" > gpurun_out/r6n_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/r6n_pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/r6_trace_cold.sh r6n pre: pre0:nav-slam_amd/lib/variants/libnavgpu_pre0.so bb1k:nav-slam_amd/lib/variants/libnavgpu_bb1k.so bbu8:nav-slam_amd/lib/variants/libnavgpu_bbu8.so pre2: pre02:nav-slam_amd/lib/variants/libnavgpu_pre0.so
