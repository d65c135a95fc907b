export NAVSLAM_QUIET=1
NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_fkey.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "knn and not mode1 and not mode3" > gpurun_out/r6f_pytest.log 2>&1; echo pytest rc=$?; tail -2 gpurun_out/r6f_pytest.log
bash scripts/r6_trace_ab.sh r6f base: fkey:nav-slam_amd/lib/variants/libnavgpu_fkey.so fkb4:nav-slam_amd/lib/variants/libnavgpu_fkb4.so base2: fkey2:nav-slam_amd/lib/variants/libnavgpu_fkey.so
bash scripts/r6_ab.sh r6f 2 "base:NAVGPU_KNN_MODE=2" "fkey:NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_fkey.so" "fkb4:NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_fkb4.so"
