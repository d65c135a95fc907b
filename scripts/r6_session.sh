export NAVSLAM_QUIET=1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "knn" > gpurun_out/r6m_pytest.log 2>&1; rc=$?; echo pytest rc=$rc; tail -2 gpurun_out/r6m_pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/r6_trace_ab.sh r6m nb2: nb1:nav-slam_amd/lib/variants/libnavgpu_nb1.so nb2b: nb1b:nav-slam_amd/lib/variants/libnavgpu_nb1.so
bash scripts/r6_ab.sh r6m 2 "nb2:NAVGPU_KNN_MODE=2" "nb1:NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_nb1.so"
