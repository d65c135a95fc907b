#!/bin/bash
# r4: K4 / K2 row screen, f32 vs f64: kernel traces and SQ counter passes
TAG=${1:-r4s7}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 PYTHONUNBUFFERED=1 TMPDIR=/tmp
Q="--no-cpu-baseline --no-traffic-json --no-stream-copy"
for w in k4 k2; do for f in 1 0; do
  NAVGPU_SCREEN_F32=$f timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d "$OUT/tr_${w}_$f" -o run \
    --output-format csv -- python3 bench.py --workload $w --steps 5 --warmup 2 $Q > "$OUT/tr_${w}_$f.log" 2>&1; rc=$?
  echo "trace $w f32=$f rc=$rc"; [ $rc -ne 0 ] && exit $rc
  NAVGPU_SCREEN_F32=$f timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
    SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU -d "$OUT/sq_${w}_$f" -o run \
    --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 $Q > "$OUT/sq_${w}_$f.log" 2>&1; rc=$?
  echo "sq $w f32=$f rc=$rc"; [ $rc -ne 0 ] && exit $rc
done; done
python3 - "$OUT" <<'PY'
import collections, csv, glob, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "tr_*", "**", "*kernel_stats.csv"), recursive=True)):
    print("==", f.split("/")[2])
    for r in csv.DictReader(open(f)):
        if float(r["Percentage"]) > 1:
            print(f"   {r['Name'].split('(')[0][-40:]:40s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
for f in sorted(glob.glob(os.path.join(o, "sq_*", "**", "*counter_collection.csv"), recursive=True)):
    agg, n = collections.defaultdict(lambda: collections.defaultdict(float)), collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    print("==", f.split("/")[2])
    for k, v in agg.items():
        if "screen" in k or "rows_match" in k or "curv" in k:
            print("  ", k, {c: round(x / len(n[k])) for c, x in v.items()})
PY
