#!/bin/bash
# r3 A/B: the product build and variants (lib/variants/libnavgpu_<v>.so),
# interleaved ROUNDS times on one box, isolated K3 k-NN times
TAG=${1:-ab}; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
for r in $(seq ${ROUNDS:-2}); do
  for v in base ${VARIANTS}; do
    lib=""; [ "$v" != base ] && lib="--lib nav-slam_amd/lib/variants/libnavgpu_$v.so"
    timeout -k 10 300 python3 scripts/knn_sweep.py $lib ${CFG:-SX=4} >> "$OUT/ab.log" 2>&1; rc=$?
    if fatal $rc; then echo "rc=$rc"; exit $rc; fi
  done
done
grep -v amdgpu.ids "$OUT/ab.log" | python3 -c "
import json,sys,collections
d=collections.defaultdict(list)
for l in sys.stdin:
    try: j=json.loads(l)
    except Exception: print(l.strip()); continue
    d[j['lib']].append((j['query_us'], j['build_us'], j['slow']))
for k,v in d.items(): print(k, v)
"
