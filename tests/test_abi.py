"""CPU-side checks of the drop-in boundary: the C-ABI libraries load and
export every symbol the headers declare, the drop-in structs keep the
reference layout, and the product fails loudly without a GPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT

INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "nav-slam_amd", "lib")


def declared(header, prefix=None):
    src = open(os.path.join(INC, header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \t\*]*?\b(\w+)\s*\(", src, flags=re.M)
    names = [n for n in names if n not in ("if", "while", "sizeof")]
    if prefix:
        names = [n for n in names if n.startswith(prefix)]
    return sorted(set(names))


def test_navgpu_exports_every_declared_symbol():
    names = declared("navgpu.h", "navgpu_")
    assert len(names) >= 25
    lib = C.CDLL(os.path.join(LIBDIR, "libnavgpu.so"))
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the python binding declares exactly these
    from navslam.gpu import exported_symbols
    assert exported_symbols() == names


@pytest.mark.parametrize("dims", ["8x8", "54x42", "64x512", "128x2048"])
def test_shim_exports_reference_api(dims):
    lib = C.CDLL(os.path.join(LIBDIR, f"libnavslam_{dims}.so"))
    names = declared("slam.h") + declared("kdtree.h") + declared("pointcloud.h")
    expect = {"init_slam", "slam_localization", "slam_mapping", "buildKDTree",
              "freeKDTree", "nearestNeighborSearch", "printKDTree",
              "convertToPointCloud", "printPointCloud"}
    extensions = {"navslam_context", "navslam_last_frame_stats"}  # not in the reference
    assert set(names) == expect | extensions
    for n in sorted(expect | extensions) + ["extract_feature"]:
        assert hasattr(lib, n), n


PROBE = r'''
#include <stddef.h>
#include <stdio.h>
#include "slam.h"
#include "ekf_probe.h"
int main(void) {
    printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(Point), sizeof(Pos),
           sizeof(KDNode), sizeof(NeighborResult), sizeof(PointCloud),
           sizeof(SLAM_attr), offsetof(SLAM_attr, kdtree_lastframe),
           offsetof(SLAM_attr, error));
    return 0;
}
'''


@pytest.mark.parametrize("R,Cc", [(8, 8), (54, 42), (128, 2048)])
def test_struct_layout_matches_reference(tmp_path, R, Cc):
    (tmp_path / "ekf_probe.h").write_text("")
    (tmp_path / "p.c").write_text(PROBE)
    exe = tmp_path / "p"
    subprocess.run(["gcc", "-std=gnu11", f"-DMAX_ROWS={R}", f"-DMAX_COLS={Cc}",
                    f"-I{INC}", f"-I{tmp_path}", str(tmp_path / "p.c"), "-o", str(exe)],
                   check=True)
    got = list(map(int, subprocess.run([str(exe)], capture_output=True, text=True,
                                       check=True).stdout.split()))
    pc = 8 + R * Cc * 24                      # int + pad + Point grid
    frame_off = 100 * pc                      # frameCount
    kd_off = (frame_off + 4 + 7) // 8 * 8     # KDNode*[R]
    err_off = kd_off + 8 * R
    assert got == [24, 48, 40, 56, pc, err_off + 8, kd_off, err_off]
    if (R, Cc) == (8, 8):
        assert got[5] == 154480


def test_reference_headers_compile_identically(tmp_path):
    """When the reference is present, our headers give its exact layout."""
    ref = "/root/reference"
    if not os.path.isdir(ref):
        pytest.skip("reference not mounted")
    (tmp_path / "ekf_probe.h").write_text("")
    (tmp_path / "p.c").write_text(PROBE)
    outs = []
    for inc in ([f"-I{INC}"], [f"-I{ref}/headers", f"-I{ref}/utils"]):
        exe = tmp_path / f"p{len(outs)}"
        subprocess.run(["gcc", "-std=gnu11", *inc, f"-I{tmp_path}", str(tmp_path / "p.c"),
                        "-o", str(exe)], check=True)
        outs.append(subprocess.run([str(exe)], capture_output=True, text=True).stdout)
    assert outs[0] == outs[1]


def test_product_has_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from navslam.gpu import NavGpu, NavGpuError
    with pytest.raises(NavGpuError):
        NavGpu(0)


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "nav-slam_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".c", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dp, f), errors="replace").read()
                assert "pyoracle" not in txt and "liboracle" not in txt \
                    and "oracle.h" not in txt, f
