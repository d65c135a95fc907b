"""PCIe copy probe for the K5 frame (r5): per-call times of the frame's
6.3 MB host<->device copies, with the host side (a) one fixed buffer,
(b) rotating over 8 source clouds / 100 map slots as the K5 loop does,
(c) a page-locked buffer, (d) a host memcpy of the same size, and (e)
pageable downloads into calloc'd slots whole and in pieces of 0.5-5 MB
(issued here as separate navgpu_download calls). The page-locked
bounce-buffer path it also timed in r5 was removed from the library after
losing (profiles/r5/copy_probe_staged.json).
Prints one JSON line. GPU only."""
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
    nb = 24 * 128 * 2048
    g = NavGpu()
    L, h = g.L, g.h
    d = C.c_void_p()
    assert L.navgpu_malloc(h, nb, C.byref(d)) == 0
    src = [np.random.rand(nb // 8) for _ in range(8)]
    slots = np.zeros((100, nb // 8))  # touched
    slots += 1.0
    pin = C.c_void_p()
    assert L.navgpu_host_alloc(h, nb, C.byref(pin)) == 0
    C.memset(pin, 0, nb)
    out = {}

    def timeit(name, fn, reps=40):
        for i in range(3):
            fn(i)
        L.navgpu_sync(h)
        ts = []
        for i in range(reps):
            t0 = time.perf_counter()
            fn(i)
            L.navgpu_sync(h)
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts) * 1e3
        out[name] = {"ms_med": round(float(np.median(ts)), 4), "ms_mean": round(float(ts.mean()), 4),
                     "ms_max": round(float(ts.max()), 4)}

    timeit("h2d_fixed", lambda i: L.navgpu_upload(h, d, src[0].ctypes.data, nb))
    timeit("h2d_rot8", lambda i: L.navgpu_upload(h, d, src[i % 8].ctypes.data, nb))
    timeit("h2d_pinned", lambda i: L.navgpu_upload(h, d, pin, nb))
    timeit("h2d_rot8_sync_each", lambda i: L.navgpu_upload(h, d, src[(3 * i) % 8].ctypes.data, nb))
    timeit("d2h_fixed", lambda i: L.navgpu_download(h, slots[0].ctypes.data, d, nb))
    timeit("d2h_rot100", lambda i: L.navgpu_download(h, slots[(7 * i) % 100].ctypes.data, d, nb))
    timeit("d2h_pinned", lambda i: L.navgpu_download(h, pin, d, nb))
    pin_np = np.ctypeslib.as_array(C.cast(pin, C.POINTER(C.c_double)), shape=(nb // 8,))
    timeit("memcpy_pin_to_slot", lambda i: np.copyto(slots[(7 * i) % 100], pin_np))
    timeit("memcpy_src_to_pin", lambda i: np.copyto(pin_np, src[i % 8]))
    # the K5 caller's map: a ctypes (calloc'd, 4 KB pages) array of slots
    cslots = (C.c_double * (100 * (nb // 8)))()
    C.memset(cslots, 1, C.sizeof(cslots))
    cbase = C.addressof(cslots)
    timeit("d2h_crot100", lambda i: L.navgpu_download(h, cbase + ((7 * i) % 100) * nb, d, nb))
    timeit("h2d_crot8", lambda i: L.navgpu_upload(h, d, cbase + ((3 * i) % 8) * nb, nb))
    for kb in (512, 1024, 1536, 2048, 3072, 3584, 4096, 5120):
        ch = kb << 10

        def dl_chunks(i, ch=ch):
            b = cbase + ((7 * i) % 100) * nb
            for o in range(0, nb, ch):
                L.navgpu_download(h, b + o, d.value + o, min(ch, nb - o))

        def ul_chunks(i, ch=ch):
            b = cbase + ((3 * i) % 8) * nb
            for o in range(0, nb, ch):
                L.navgpu_upload(h, d.value + o, b + o, min(ch, nb - o))

        timeit(f"d2h_crot100_{kb}k", dl_chunks)
        timeit(f"h2d_crot8_{kb}k", ul_chunks)

    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
