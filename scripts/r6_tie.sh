#!/bin/bash
# r6 tie-pass session: tree/rows parity with the chain-mode build, then
# interleaved K2i / K4i bench lines against variant libraries.
# usage: scripts/r6_tie.sh TAG ROUNDS [variant ...]   (variant: nav-slam_amd/lib/variants/libnavgpu_<v>.so)
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "${TESTS:-kd_build or rows or lazy or shim_l9 or k5_exact}" > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
fi
for r in $(seq 1 "$ROUNDS"); do
  for v in default "$@"; do
    lib=""; [ "$v" != default ] && lib="NAVGPU_LIB=nav-slam_amd/lib/variants/libnavgpu_$v.so"
    for w in ${WORKLOADS:-k2 k4}; do
      f="$OUT/${w}i_${v}_$r.json"
      env $lib timeout -k 10 300 python3 bench.py --workload $w --integer-mm --no-cpu-baseline --no-stream-copy \
        --json-out "$f" > "$OUT/${w}i_${v}_$r.log" 2>&1
      rc=$?; if [ $rc -ne 0 ]; then echo "$w $v rc=$rc"; tail -5 "$OUT/${w}i_${v}_$r.log"; exit $rc; fi
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],4), d['value'])" "$f" "$w" "$v"
    done
  done
done
