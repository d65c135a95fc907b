for v in st_base st_btw1024 st_btw8192; do timeout -k 10 120 python3 scripts/rows_probe.py --integer --lib nav-slam_amd/lib/variants/libnavgpu_$v.so || exit 1; done
SKIP_TESTS=1 WORKLOADS="k2 k4" bash scripts/r6_tie.sh r6t10 2 btw512 btw1024 btw8192
