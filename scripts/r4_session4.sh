#!/bin/bash
# r4: variant probes (k_knnw knobs, binning knobs: query_us / build_us per
# library, interleaved rounds), then SQ counter passes: K3 k_knnw and the K4
# row screen with the f32 pre-screen on and off
TAG=${1:-r4s4}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1
echo "== k_knnw variants"; VDIR=nav-slam_amd/lib/variants bash scripts/r4_var.sh "$TAG/vw" "${ROUNDS:-2}" || exit $?
echo "== binning variants"; VDIR=nav-slam_amd/lib/var_bin bash scripts/r4_var.sh "$TAG/vb" "${ROUNDS:-2}" || exit $?
[ -n "$NO_PMC" ] && exit 0
bash scripts/pmc_sq.sh "$TAG/sq_k3" || exit $?
export TMPDIR=/tmp
for f in 1 0; do
  NAVGPU_SCREEN_F32=$f timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
    SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d "$OUT/sq_k4_$f" -o run --output-format csv -- python3 bench.py \
    --workload k4 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic-json --no-stream-copy \
    > "$OUT/sq_k4_$f.log" 2>&1; rc=$?
  echo "sq_k4 f32=$f rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "sq_k4_*", "**", "*counter_collection.csv"), recursive=True)):
    agg, n = collections.defaultdict(lambda: collections.defaultdict(float)), collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        if "screen" in k or "rows_match" in k:
            print(f.split("/")[-4] if "/" in f else f, k, {c: round(x / len(n[k])) for c, x in v.items()})
PY
true
