"""K5 mapping-call sequence probe (r5): per-call host time of
upload(cloud) -> transform -> download(map slot) with calloc'd (4 KB-page)
host buffers as the K5 caller has them, in variants that separate where the
time goes, and a page-locked stage copied out by 1-8 host threads (the
bounce path DESIGN.md §4 r5 measured and dropped). Prints one JSON line.
GPU only."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
from navslam.gpu import NavGpu  # noqa: E402


def main():
    npts = 128 * 2048
    nb = 24 * npts
    g = NavGpu()
    L, h = g.L, g.h
    din, dout = C.c_void_p(), C.c_void_p()
    assert L.navgpu_malloc(h, nb, C.byref(din)) == 0
    assert L.navgpu_malloc(h, nb, C.byref(dout)) == 0
    src = (C.c_double * (8 * npts * 3))()
    slots = (C.c_double * (100 * npts * 3))()
    C.memset(slots, 0, C.sizeof(slots))
    rng = np.random.default_rng(0)
    np.ctypeslib.as_array(src)[:] = rng.random(8 * npts * 3) * 1000
    sb, db = C.addressof(src), C.addressof(slots)
    Rm = np.eye(3)
    t = np.zeros(3)
    out = {}

    def up(i):
        L.navgpu_upload(h, din, sb + (i % 8) * nb, nb)

    def tf(i):
        g.transform_dev(din.value, npts, Rm, t, None, dout.value)

    def down(i):
        L.navgpu_download(h, db + ((7 * i) % 100) * nb, dout, nb)

    def sync(i):
        L.navgpu_sync(h)

    def run(name, seq, reps=60):
        for i in range(5):
            for f in seq:
                f(i)
            sync(i)
        ts = []
        for i in range(reps):
            t0 = time.perf_counter()
            for f in seq:
                f(i)
            sync(i)
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts) * 1e3
        out[name] = {"ms_med": round(float(np.median(ts)), 4), "ms_mean": round(float(ts.mean()), 4)}

    run("up", [up])
    run("tf", [tf])
    run("down", [down])
    run("up_tf_down", [up, tf, down])
    run("up_tf_sync_down", [up, tf, sync, down])
    run("up_sync_tf_sync_down", [up, sync, tf, sync, down])
    # page-locked stage + parallel host copy-out (ctypes.memmove drops the GIL)
    from concurrent.futures import ThreadPoolExecutor
    pin = C.c_void_p()
    assert L.navgpu_host_alloc(h, nb, C.byref(pin)) == 0
    C.memset(pin, 0, nb)
    for T in (1, 2, 4, 8):
        ex = ThreadPoolExecutor(T)
        part = (nb // T + 4095) & ~4095

        def copy_out(i, T=T, part=part, ex=ex):
            dst = db + ((7 * i) % 100) * nb
            fs = [ex.submit(C.memmove, dst + o, pin.value + o, min(part, nb - o))
                  for o in range(0, nb, part)]
            for f in fs:
                f.result()

        def dl_pin(i):
            L.navgpu_download(h, pin, dout, nb)
            L.navgpu_sync(h)

        run(f"memcpy_out_T{T}", [copy_out])
        run(f"dl_pin_then_copy_T{T}", [dl_pin, copy_out])
        ex.shutdown()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
