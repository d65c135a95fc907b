"""SURVEY.md §5 "ASan/UBSan on the host restatement" (CPU only).

oracle/Makefile `asan` builds, under -fsanitize=address,undefined with
-fno-sanitize-recover (any report aborts the program):
  * oracle_asan        oracle/asan_driver.c over the oracle restatement
                       (oracle.c, oracle_grid.c) and the jansson subset
                       (nav-slam_amd/jansson/jansson_mini.c), on edge inputs:
                       empty / single-point / duplicate / NaN trees, rows
                       without features, k > n, hostile JSON;
  * shim_asan_54x42    the drop-in shim's host half (nav-slam_amd/csrc/
                       navslam_shim.c: KDNode slabs and registry, list
                       download, exact and fast Adam tails, host trees on and
                       off) over oracle/navgpu_cpu_stub.c, a host stand-in
                       for libnavgpu: 130 frames through the 100-frame map
                       ring, exact-mode poses bit-identical to the oracle's
                       frame loop, plus buildKDTree / nearestNeighborSearch /
                       freeKDTree on a point set and a caller-linked tree;
  * nav_slam_ref_8x8, nav_slam_l9_ref_8x8 (with /root/reference): the K1
                       reference programs, whose L5 JSON and L9 CSV readers
                       (src/main.c:13-128) run over our jansson subset, fed the
                       same L5 JSON and L9 CSV fixtures as tests/test_k1_main.py.
"""
import os
import subprocess

import pytest

from conftest import ROOT

ASAN = os.path.join(ROOT, "oracle", "_asan")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="2")
ENV.pop("NAVSLAM_QUIET", None)
REPORTS = ("ERROR: AddressSanitizer", "runtime error:", "ERROR: LeakSanitizer")


@pytest.fixture(scope="module")
def built():
    p = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"],
                       capture_output=True, text=True)
    if p.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + p.stdout[-2000:] + p.stderr[-2000:])
    return ASAN


def _clean(p):
    err = p.stderr.decode(errors="replace") if isinstance(p.stderr, bytes) else p.stderr
    assert p.returncode == 0, err[-3000:]
    for r in REPORTS:
        assert r not in err, err[-3000:]


def test_oracle_and_jansson_under_asan_ubsan(built):
    p = subprocess.run([os.path.join(built, "oracle_asan")], env=ENV, capture_output=True,
                       text=True, timeout=600)
    _clean(p)
    assert "asan_driver ok" in p.stdout


def test_shim_host_code_under_asan_ubsan(built):
    p = subprocess.run([os.path.join(built, "shim_asan_54x42")], env=ENV, capture_output=True,
                       text=True, timeout=600)
    _clean(p)
    assert "shim_asan ok" in p.stdout


def _exe(built, name):
    path = os.path.join(built, name)
    if not os.path.exists(path):
        pytest.skip(f"{path} not built (needs /root/reference)")
    return path


def test_k1_l5_json_reader_under_asan(built, tmp_path):
    from test_k1_main import l5_json, stream
    depth, imu, ts = stream(8, 8, 10, seed=5)
    l5_json(str(tmp_path / "parsed_data.json"), depth, imu, ts)
    p = subprocess.run([_exe(built, "nav_slam_ref_8x8")], cwd=str(tmp_path), env=ENV,
                       capture_output=True, timeout=600)
    _clean(p)
    with open(tmp_path / "point_cloud_data.csv") as fh:
        assert len(fh.read().splitlines()) == 1 + 10 * 8 * 8


def test_k1_l9_csv_reader_under_asan(built, tmp_path):
    from test_k1_main import l9_frames
    fr = l9_frames(8, 8, 6, seed=4)
    F, R, Cc, _ = fr.shape
    lines = ["frame,row,col,x,y,z,conf"]
    for f in range(F):
        for r in range(R):
            for c in range(Cc):
                x, y, z = fr[f, r, c]
                lines.append(f"{f},{r},{c},{x},{y},{z},{(r * 7 + c) % 100}")
    (tmp_path / "parsed_data.csv").write_text("\n".join(lines) + "\n")
    p = subprocess.run([_exe(built, "nav_slam_l9_ref_8x8")], cwd=str(tmp_path), env=ENV,
                       capture_output=True, timeout=600)
    _clean(p)
    with open(tmp_path / "point_cloud_data.csv") as fh:
        assert len(fh.read().splitlines()) == 1 + F * R * Cc
