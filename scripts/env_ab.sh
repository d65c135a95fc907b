#!/bin/bash
# K3 bench.py A/B over environment variants, interleaved rounds on one box:
#   scripts/env_ab.sh OUTDIR ROUNDS "VAR=a VAR2=b" "VAR=c" ...
# prints ms_per_step and the isolated kernel times per variant and round.
OUT=gpurun_out/$1; ROUNDS=$2; shift 2; mkdir -p "$OUT"
for r in $(seq "$ROUNDS"); do
  for v in "$@"; do
    env $v timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline \
      --no-stream-copy ${BENCH_ARGS} --json-out "$OUT/b.json" > "$OUT/b.log" 2>&1 || { tail -20 "$OUT/b.log"; exit 1; }
    python3 - "$v" "$OUT/b.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(f"{sys.argv[1]:28s}", d["ms_per_step"], d["kernel_us_isolated"], flush=True)
PY
  done
done
