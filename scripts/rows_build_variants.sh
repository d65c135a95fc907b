#!/bin/bash
# k_rows_build probe over the product library and any variants given
# (names under nav-slam_amd/lib/variants/libnavgpu_<name>.so); optional
# pytest -k filter first (PYTEST_K)
set -e
OUT=gpurun_out/${TAG:-rb}; mkdir -p "$OUT"
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method=thread -k "$PYTEST_K" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
  grep -E "passed|failed" "$OUT/pytest.log" | tail -1
fi
for v in default "$@"; do
  L=""; [ "$v" != default ] && L="--lib nav-slam_amd/lib/variants/libnavgpu_$v.so"
  timeout -k 10 120 python3 scripts/rows_build_probe.py $L --tag "$v" >> "$OUT/out.jsonl"
done
cat "$OUT/out.jsonl"
