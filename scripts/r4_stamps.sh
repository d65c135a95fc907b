#!/bin/bash
# r4: k_knnw phase stamps (per-wave records, summed) on the K3 probe
OUT=gpurun_out/${1:-r4st}; mkdir -p "$OUT"
NAVGPU_KNN_MODE=1 timeout -k 10 120 python3 scripts/knn_probe.py --occ 5 --reps 5 \
  --lib ${LIB:-nav-slam_amd/lib/variants/libnavgpu_stamps.so} > "$OUT/probe.json" 2>&1 || { cat "$OUT/probe.json"; exit 1; }
python3 - "$OUT/probe.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["stamps"]["raw"]; n = max(r[1], 1)
print("query_us", round(d["query_us"], 1), "chunks", r[1], "rounds/chunk", r[7] / n)
for i, nm in [(2, "tables"), (3, "staging"), (4, "scan(l0)"), (6, "next tables"), (5, "exact(l0)"),
              (8, "wave lifetime / chunks")]:
    print(f"{nm:24s} {r[i] / n:10.0f} cycles per chunk")
PY
