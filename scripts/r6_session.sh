export NAVSLAM_QUIET=1; mkdir -p gpurun_out/r6j
timeout -k 10 120 python3 scripts/knng_timeline.py --lib nav-slam_amd/lib/variants/libnavgpu_pstamps.so > gpurun_out/r6j/timeline_pers.json 2>gpurun_out/r6j/timeline.err; echo tl rc=$?; cat gpurun_out/r6j/timeline_pers.json
