"""bench.py's measurement plumbing on the CPU: the per-step HBM bytes taken
from rocprofv3 --pmc counter CSVs (FETCH_SIZE x2 + WRITE_SIZE, per launch of
the workload's anchor kernel), the per-workload traffic json lookup, and the
json scripts/traffic_json.py writes from two such passes."""
import argparse
import csv
import json
import os
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _pmc_csv(path, counter, rows):
    """rows: (dispatch id, kernel name, value in KB)"""
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name",
                                          "Counter_Value"])
        w.writeheader()
        for d, name, v in rows:
            w.writerow({"Dispatch_Id": d, "Kernel_Name": name, "Counter_Name": counter,
                        "Counter_Value": v})


def _k3_passes(tmp_path, main="k_knnw"):
    knn = f"void (anonymous namespace)::{main}<8>((anonymous namespace)::GridParams const*)"
    slow = "void (anonymous namespace)::k_knn_slow<8>(int)"
    hist = "(anonymous namespace)::k_bin_hist((anonymous namespace)::BinJob)"
    f, w = str(tmp_path / "fetch.csv"), str(tmp_path / "write.csv")
    # two steps: the query pass launched once per step
    _pmc_csv(f, "FETCH_SIZE", [(1, hist, 10), (2, knn, 100), (3, slow, 4),
                               (4, hist, 12), (5, knn, 102), (6, slow, 2)])
    _pmc_csv(w, "WRITE_SIZE", [(1, hist, 1), (2, knn, 50), (3, slow, 1),
                               (4, hist, 3), (5, knn, 52), (6, slow, 1)])
    return f, w


import pytest  # noqa: E402


@pytest.mark.parametrize("main", ["k_knnw", "k_knng"])
def test_pmc_bytes_per_step(tmp_path, main):
    """k_knnw (NAVGPU_KNN_MODE=1) or k_knng (2) is the per-step anchor."""
    f, w = _k3_passes(tmp_path, main)
    q = bench.pmc_bytes([f, w], bench.QUERY_KERNELS)
    # fetch (100+4+102+2)/2 = 104 KB, write (50+1+52+1)/2 = 52 KB
    assert q == {"fetch_raw": 104 * 1024, "write": 52 * 1024, "bytes": (2 * 104 + 52) * 1024}
    b = bench.pmc_bytes([f, w], bench.BUILD_KERNELS)
    assert b == {"fetch_raw": 11 * 1024, "write": 2 * 1024, "bytes": (2 * 11 + 2) * 1024}
    assert bench.traffic_from_csv([f, w]) == q["bytes"]
    # no anchor launches: no per-step figure
    assert bench.pmc_bytes([f, w], bench.QUERY_KERNELS, anchor="k_rows_screen") is None


def test_traffic_json_script_and_lookup(tmp_path):
    f, w = _k3_passes(tmp_path)
    out = tmp_path / "traffic_k3.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "traffic_json.py"), f, w,
                    str(out), "t", "--workload", "k3"], check=True, capture_output=True)
    rec = json.loads(out.read_text())
    assert rec["bytes_per_step"] == (2 * 104 + 52) * 1024
    assert rec["build_bytes_per_step"] == (2 * 11 + 2) * 1024
    a = argparse.Namespace(workload="k3", integer_mm=False, k5_mode="exact",
                           no_traffic_json=False, traffic_json=str(out))
    assert bench.traffic_tag(a) == "k3"
    assert bench.load_traffic(a, {"k": 8, "points_per_cloud": 1048576}) == rec
    assert bench.load_traffic(a, {"k": 4, "points_per_cloud": 1048576}) is None
    a.no_traffic_json = True
    assert bench.load_traffic(a, {"k": 8}) is None


def test_traffic_tags(monkeypatch):
    ns = lambda **kw: argparse.Namespace(**dict(dict(integer_mm=False, k5_mode="exact"), **kw))
    assert bench.traffic_tag(ns(workload="k2", integer_mm=True)) == "k2i"
    assert bench.traffic_tag(ns(workload="k4")) == "k4"
    monkeypatch.delenv("NAVSLAM_HOST_TREES", raising=False)
    assert bench.traffic_tag(ns(workload="k5", k5_mode="fast")) == "k5f"
    # fast mode with lazy row trees quotes its own PMC bytes (r6)
    monkeypatch.setenv("NAVSLAM_HOST_TREES", "0")
    assert bench.traffic_tag(ns(workload="k5", k5_mode="fast")) == "k5fl"
    assert bench.traffic_tag(ns(workload="k5")) == "k5"
    with open(os.path.join(ROOT, "profiles", "traffic_k5fl.json")) as fh:
        tl = json.load(fh)
    assert tl["workload"] == "k5fl" and tl["points_per_cloud"] == 128 * 2048
    assert tl["bytes_per_step"] > 0
    # the default bench line reads the committed K3 json, which must match its config
    with open(os.path.join(ROOT, "profiles", "traffic_k3.json")) as fh:
        tj = json.load(fh)
    assert tj["k"] == 8 and tj["points_per_cloud"] == 1048576 and tj["bytes_per_step"] > 0
