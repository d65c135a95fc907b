"""K3 build and query times on a CU-masked stream (r5 probe): how the index
build and the query pass scale with the CUs they may use. Prints one JSON
line per mask. GPU only."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))
import torch  # noqa: E402

from navslam import synth  # noqa: E402
from navslam.gpu import NavGpu  # noqa: E402


def hip_lib():
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                return C.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not loaded")


def main():
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    H = hip_lib()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    s, t = synth.uniform_pair(512, 2048)
    N = s.shape[0] * s.shape[1]
    src = torch.from_numpy(s).to(dev)
    tgt = torch.from_numpy(t).to(dev)
    idx = torch.empty((N, 8), dtype=torch.int32, device=dev)
    dst = torch.empty((N, 8), dtype=torch.float64, device=dev)
    masks = [("all", lambda c: True), ("1of8", lambda c: c % 8 == 0),
             ("low64", lambda c: c < 64), ("low128", lambda c: c < 128),
             ("high128", lambda c: c >= 128), ("low192", lambda c: c < 192),
             ("high64", lambda c: c >= 192)]
    masks += [(f"blk32_{k}", lambda c, k=k: 32 * k <= c < 32 * k + 32) for k in (0, 1, 7)]
    masks += [("mod32lt8", lambda c: c % 32 < 8), ("mod32lt16", lambda c: c % 32 < 16),
              ("mod32lt24", lambda c: c % 32 < 24)]
    for name, keep in masks:
        words = [0] * ((ncu + 31) // 32)
        for c in range(ncu):
            if keep(c):
                words[c // 32] |= 1 << (c % 32)
        arr = (C.c_uint32 * len(words))(*words)
        st = C.c_void_p()
        rc = H.hipExtStreamCreateWithCUMask(C.byref(st), len(words), arr)
        if rc != 0:
            print(json.dumps({"mask": name, "error": rc}), flush=True)
            continue
        g = NavGpu(0, st.value)
        g.knn_dev(tgt, N, src, N, 8, idx, dst)
        g.sync()
        g.timing(True)
        for _ in range(10):
            g.knn_dev(tgt, N, src, N, 8, idx, dst)
        g.sync()
        q_ms, qn = g.timing_read("knn_query")
        b_ms, bn = g.timing_read("knn_build")
        print(json.dumps({"mask": name, "cus": sum(bin(w).count("1") for w in words),
                          "build_us": round(1000 * b_ms / bn, 1),
                          "query_us": round(1000 * q_ms / qn, 1)}), flush=True)
        g.close()
        H.hipStreamDestroy(st)


if __name__ == "__main__":
    main()
