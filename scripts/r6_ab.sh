#!/bin/bash
# Interleaved K3 bench A/B on one box: r6_ab.sh TAG ROUNDS "label:ENV=V ENV2=V[@bench args]" ...
# Each arm: python3 bench.py with that env (plus $BENCH_ARGS); one summary line per run.
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    label=${spec%%:*}; rest=${spec#*:}
    envs=${rest%%@*}; args=""; [ "$rest" != "$envs" ] && args=${rest#*@}
    f="$OUT/${label}_$r.json"
    env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-stream-copy $BENCH_ARGS $args --json-out "$f" > "$OUT/${label}_$r.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$label round $r rc=$rc"; tail -5 "$OUT/${label}_$r.log"; exit $rc; fi
    python3 scripts/k3_line_summary.py "$label" "$f"
  done
done
