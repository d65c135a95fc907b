#!/bin/bash
# k-NN iteration session: k-NN GPU parity tests, the probe (query/build us),
# and the LDS/VALU SQ counter pass over the probe
TAG=${1:-kq}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export NAVSLAM_QUIET=1 NAVGPU_KNN_STATS=1 TMPDIR=/tmp
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
PYTHONUNBUFFERED=1 timeout -k 10 600 python3 -m pytest tests -m gpu -v -x --timeout 240 --timeout-method=thread -k "${PYTEST_K:-knn}" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc $(tail -n 1 $OUT/pytest.log)"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python3 scripts/knn_probe.py --occ ${OCC:-5} --reps 20 > "$OUT/probe.log" 2>&1; rc=$?
echo "probe rc=$rc $(grep query_us $OUT/probe.log | cut -c1-160)"; if fatal $rc; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d "$OUT/pmc" -o run --output-format csv -- python3 scripts/knn_probe.py --occ 5 --reps 2 > "$OUT/pmc.log" 2>&1; rc=$?
echo "pmc rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python3 scripts/pmc_summary.py "$OUT" | grep -A1 "k_knn<8, false" | cut -c1-400
