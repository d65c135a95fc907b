#!/bin/bash
# k_bbox_partial block size 1024/512/256: k-NN tests, then K3 A/B against HEAD's build (variants/old)
OUT=gpurun_out/$1; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1 NAVSLAM_QUIET=1
D=nav-slam_amd/lib/variants/old
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "knn or global or k3 or golden" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for r in 1 2 3; do
  for v in "NAVGPU_X=new1024" "NAVGPU_LIB=nav-slam_amd/lib/variants/x/libnavgpu_t512.so" "NAVGPU_LIB=nav-slam_amd/lib/variants/x/libnavgpu_t256.so"; do
    env $v timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-traffic-json --no-stream-copy --json-out "$OUT/k3.json" > "$OUT/k3.log" 2>&1 || { tail "$OUT/k3.log"; exit 1; }
    python3 scripts/k3_line_summary.py "${v: -12}" "$OUT/k3.json"
  done
done
export TMPDIR=/tmp
for L in "" nav-slam_amd/lib/variants/x/libnavgpu_t512.so nav-slam_amd/lib/variants/x/libnavgpu_t256.so; do
  T="$OUT/trace_$(basename "${L:-new}" .so)"
  NAVGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$T" -o run --output-format csv -- python3 bench.py --inflight 1 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic-json --no-stream-copy > "$OUT/trace.log" 2>&1 || exit 1
  echo "$T: $(grep -h k_bbox_partial $(find "$T" -name "*kernel_stats.csv") | cut -d, -f2-5)"
done
