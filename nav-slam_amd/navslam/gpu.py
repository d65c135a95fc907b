"""ctypes binding of libnavgpu.so (include/navgpu.h).

The HIP library is the product: if it is missing or the device is not a
gfx950 the constructor raises — there is no CPU fallback anywhere in this
package. Host-pointer calls take/return numpy arrays; device-pointer calls
take torch tensors (or raw integer addresses) already resident on the GPU.
"""
import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.abspath(os.path.join(PKG, "..", "lib"))
# NAVGPU_LIB: an experimental build of the same library (A/B runs only)
LIBNAVGPU = os.environ.get("NAVGPU_LIB") or os.path.join(LIBDIR, "libnavgpu.so")

NAVGPU_OK = 0

_vp = C.c_void_p
_i32 = C.c_int32
_sz = C.c_size_t


class NavGpuError(RuntimeError):
    pass


def _declare(L):
    sig = {
        "navgpu_create": (C.c_int, [C.c_int, _vp, C.POINTER(_vp)]),
        "navgpu_destroy": (None, [_vp]),
        "navgpu_set_stream": (C.c_int, [_vp, _vp]),
        "navgpu_stream": (_vp, [_vp]),
        "navgpu_sync": (C.c_int, [_vp]),
        "navgpu_last_error": (C.c_char_p, []),
        "navgpu_version": (C.c_char_p, []),
        "navgpu_rows_max_cols": (C.c_int, []),
        "navgpu_curvature_dev": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _vp, _vp]),
        "navgpu_curvature_host": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _vp, _vp]),
        "navgpu_project_dev": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _vp]),
        "navgpu_project_host": (C.c_int, [_vp, _vp, C.c_int, C.c_int, _vp]),
        "navgpu_transform_dev": (C.c_int, [_vp, _vp, _sz, _vp, _vp, _vp, _vp, _vp]),
        "navgpu_kd_build_rows_dev": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int,
                                               _vp, _vp, _vp, _vp]),
        "navgpu_kd_query_rows_dev": (C.c_int, [_vp, _vp, _vp, _vp, _vp, C.c_int,
                                               C.c_int, _vp, _vp, _vp]),
        "navgpu_kd_compact_rows_dev": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int,
                                                 _vp, _vp, _vp, _vp, _vp]),
        "navgpu_kd_query_rows_lazy_dev": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp,
                                                    C.c_int, C.c_int, _vp, _vp, _vp, _vp]),
        "navgpu_kd_query_rows_lazy_corr_dev": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp,
                                                         C.c_int, C.c_int, _vp, _vp, _vp, _vp,
                                                         _vp, _vp]),
        "navgpu_rows_corr_dev": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, C.c_int,
                                           C.c_int, _vp, _vp]),
        "navgpu_rows_corr_list_dev": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, C.c_int,
                                               C.c_int, _vp, _vp]),
        "navgpu_rows_match_dev": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int,
                                            _vp, _vp, _vp, _vp]),
        "navgpu_rows_match_host": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int,
                                             _vp, _vp, _vp, _vp]),
        "navgpu_rows_match_batch_dev": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int, C.c_int,
                                                  _vp, _vp, _vp, _vp]),
        "navgpu_knn_dev": (C.c_int, [_vp, _vp, _sz, _vp, _sz, C.c_int, _vp, _vp]),
        "navgpu_knn_host": (C.c_int, [_vp, _vp, _sz, _vp, _sz, C.c_int, _vp, _vp]),
        "navgpu_pair_knn_dev": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int, C.c_int,
                                          _vp, _vp, _vp, _vp]),
        "navgpu_kd_build_dev": (C.c_int, [_vp, _vp, _sz, C.c_int]),
        "navgpu_kd_build_host": (C.c_int, [_vp, _vp, _sz, C.c_int]),
        "navgpu_malloc": (C.c_int, [_vp, _sz, C.POINTER(_vp)]),
        "navgpu_free": (None, [_vp, _vp]),
        "navgpu_host_alloc": (C.c_int, [_vp, _sz, C.POINTER(_vp)]),
        "navgpu_host_free": (None, [_vp, _vp]),
        "navgpu_host_register": (C.c_int, [_vp, _vp, _sz]),
        "navgpu_host_unregister": (None, [_vp, _vp]),
        "navgpu_kd_rows_nodes_dev": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int, C.c_uint64,
                                               _vp, _vp]),
        "navgpu_upload": (C.c_int, [_vp, _vp, _vp, _sz]),
        "navgpu_download": (C.c_int, [_vp, _vp, _vp, _sz]),
        "navgpu_stream_copy_dev": (C.c_int, [_vp, _vp, _vp, _sz]),
        "navgpu_side_mark": (C.c_int, [_vp]),
        "navgpu_side_download": (C.c_int, [_vp, _vp, _vp, _sz]),
        "navgpu_timing_enable": (None, [_vp, C.c_int]),
        "navgpu_timing_select": (None, [_vp, C.c_char_p]),
        "navgpu_timing_read": (C.c_double, [_vp, C.c_char_p, C.c_int]),
        "navgpu_timing_count": (C.c_int, [_vp, C.c_char_p]),
        "navgpu_knn_fallbacks": (C.c_longlong, [_vp]),
        "navgpu_knn_overflows": (C.c_longlong, [_vp]),
        "navgpu_knn_check": (C.c_int, [_vp]),
        "navgpu_rows_tie_rows": (C.c_longlong, [_vp]),
        "navgpu_debug_nth_element": (C.c_int, [_vp, _vp, _vp, C.c_int, C.c_int, C.c_int,
                                               C.c_int, C.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return sig


_LIB = None


def load_library(path=LIBNAVGPU):
    """Load libnavgpu.so (raises if it was not built)."""
    global _LIB
    if _LIB is None:
        # Bind to the HIP runtime torch ships when torch is present: torch loads
        # its bundled libamdhip64 (SONAME libamdhip64.so.7) by path, so loading
        # /opt/rocm's copy first would leave two HSA runtimes in the process.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(path):
            raise NavGpuError(
                f"{path} is missing: build it with `make -C nav-slam_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        _LIB = C.CDLL(path)
        _declare(_LIB)
    return _LIB


def exported_symbols():
    """Names of every C entry point declared in include/navgpu.h."""
    L = load_library()
    return sorted(_declare(L).keys())


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()  # torch tensor


class NavGpu:
    """A libnavgpu context: device + stream + workspace."""

    def __init__(self, device=0, stream=None):
        self.L = load_library()
        h = _vp()
        self._check(self.L.navgpu_create(device, stream, C.byref(h)), "navgpu_create")
        self.h = h

    def _check(self, rc, what):
        if rc != NAVGPU_OK:
            msg = self.L.navgpu_last_error().decode(errors="replace")
            raise NavGpuError(f"{what} failed ({rc}): {msg}")

    def close(self):
        if getattr(self, "h", None):
            self.L.navgpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------- plumbing
    def set_stream(self, stream_handle):
        self._check(self.L.navgpu_set_stream(self.h, stream_handle), "set_stream")

    def sync(self):
        self._check(self.L.navgpu_sync(self.h), "sync")

    @property
    def rows_max_cols(self):
        return self.L.navgpu_rows_max_cols()

    def timing(self, on=True):
        self.L.navgpu_timing_enable(self.h, 1 if on else 0)

    def timing_select(self, name=None):
        """Record only the region `name` while timing is on (None: all)."""
        self.L.navgpu_timing_select(self.h, None if name is None else name.encode())

    def stream_copy_dev(self, dst, src, nbytes):
        """Device-to-device copy by a plain streaming kernel (the measured HBM
        ceiling beside the roofline's peak; timed as "stream_copy")."""
        self._check(self.L.navgpu_stream_copy_dev(self.h, _ptr(dst), _ptr(src), nbytes),
                    "stream_copy_dev")

    def knn_fallbacks(self):
        """Queries of the last knn call that took the exact slow path (-1 if
        not recorded; set NAVGPU_KNN_STATS=1 before creating the context)."""
        return self.L.navgpu_knn_fallbacks(self.h)

    def knn_overflows(self):
        """k_knn tiles of the last knn call that overflowed the LDS tile and
        ran from global memory."""
        return self.L.navgpu_knn_overflows(self.h)

    def knn_check(self):
        """Raises NavGpuError (NAVGPU_EINTERNAL) when a k-NN kernel of the last
        knn call met an out-of-range index (synchronises)."""
        self._check(self.L.navgpu_knn_check(self.h), "knn_check")

    def rows_tie_rows(self):
        """Rows of the last rows_match call that had a distance tie and ran
        the reference tree (-1 if that call did not screen)."""
        return self.L.navgpu_rows_tie_rows(self.h)

    def debug_nth_element(self, key, perm, first, last, nth, block=False):
        """One reference nth_element as the per-row builds run it (device
        tensors: key f64 [n], perm int32 [n], permuted in place)."""
        self._check(self.L.navgpu_debug_nth_element(self.h, _ptr(key), _ptr(perm), len(perm),
                                                    first, last, nth, 1 if block else 0),
                    "debug_nth_element")

    def timing_read(self, name, reset=True):
        n = self.L.navgpu_timing_count(self.h, name.encode())
        ms = self.L.navgpu_timing_read(self.h, name.encode(), 1 if reset else 0)
        return ms, n

    # ---------------------------------------------------- host-pointer API
    def curvature(self, pts, want_curv=False):
        pts = np.ascontiguousarray(pts, np.float64)
        R, Cc = pts.shape[:2]
        mask = np.zeros((R, Cc), np.int32)
        curv = np.zeros((R, Cc)) if want_curv else None
        self._check(self.L.navgpu_curvature_host(self.h, _ptr(pts), R, Cc, _ptr(mask),
                                                 _ptr(curv)), "curvature")
        return (mask, curv) if want_curv else mask

    def project(self, depth):
        depth = np.ascontiguousarray(depth, np.int32)
        R, Cc = depth.shape
        out = np.zeros((R, Cc, 3))
        self._check(self.L.navgpu_project_host(self.h, _ptr(depth), R, Cc, _ptr(out)),
                    "project")
        return out

    def rows_match(self, src, tgt):
        src = np.ascontiguousarray(src, np.float64)
        tgt = np.ascontiguousarray(tgt, np.float64)
        R, Cc = src.shape[:2]
        sm = np.zeros((R, Cc), np.int32)
        tm = np.zeros((R, Cc), np.int32)
        idx = np.zeros((R, Cc), np.int32)
        dist = np.zeros((R, Cc))
        self._check(self.L.navgpu_rows_match_host(self.h, _ptr(src), _ptr(tgt), R, Cc,
                                                  _ptr(sm), _ptr(tm), _ptr(idx), _ptr(dist)),
                    "rows_match")
        return sm, tm, idx, dist

    def knn(self, tgt, queries, k):
        tgt = np.ascontiguousarray(tgt, np.float64).reshape(-1, 3)
        q = np.ascontiguousarray(queries, np.float64).reshape(-1, 3)
        idx = np.zeros((len(q), k), np.int32)
        dist = np.zeros((len(q), k))
        self._check(self.L.navgpu_knn_host(self.h, _ptr(tgt), len(tgt), _ptr(q), len(q), k,
                                           _ptr(idx), _ptr(dist)), "knn")
        return idx, dist

    def kd_build(self, pts, depth0=0):
        """Reference buildKDTree permutation of `pts` (returns a new array)."""
        p = np.array(pts, np.float64, order="C").reshape(-1, 3)
        self._check(self.L.navgpu_kd_build_host(self.h, _ptr(p), len(p), depth0),
                    "kd_build")
        return p

    # -------------------------------------------------- device-pointer API
    def curvature_dev(self, pts, R, Cc, mask, curv=None):
        self._check(self.L.navgpu_curvature_dev(self.h, _ptr(pts), R, Cc, _ptr(mask),
                                                _ptr(curv)), "curvature_dev")

    def transform_dev(self, pts, n, Rm, t, tr, out, out_last=None):
        Rm = np.ascontiguousarray(Rm, np.float64)
        t = np.ascontiguousarray(t, np.float64)
        tr = None if tr is None else np.ascontiguousarray(tr, np.float64)
        self._check(self.L.navgpu_transform_dev(self.h, _ptr(pts), n, _ptr(Rm), _ptr(t),
                                                _ptr(tr), _ptr(out), _ptr(out_last)),
                    "transform_dev")

    def kd_build_dev(self, pts, n, depth0=0):
        self._check(self.L.navgpu_kd_build_dev(self.h, _ptr(pts), n, depth0), "kd_build_dev")

    def kd_build_rows_dev(self, feat_src, coords, R, Cc, tree_pts, tree_col, tree_n,
                          mask=None):
        self._check(self.L.navgpu_kd_build_rows_dev(
            self.h, _ptr(feat_src), _ptr(coords), R, Cc, _ptr(tree_pts), _ptr(tree_col),
            _ptr(tree_n), _ptr(mask)), "kd_build_rows_dev")

    def kd_rows_nodes_dev(self, tree_pts, tree_n, R, Cc, host_base, nodes, row_off):
        self._check(self.L.navgpu_kd_rows_nodes_dev(
            self.h, _ptr(tree_pts), _ptr(tree_n), R, Cc, int(host_base), _ptr(nodes),
            _ptr(row_off)), "kd_rows_nodes_dev")

    def kd_query_rows_dev(self, tree_pts, tree_n, feat_src, queries, R, Cc, nn_pos,
                          nn_dist, mask=None):
        self._check(self.L.navgpu_kd_query_rows_dev(
            self.h, _ptr(tree_pts), _ptr(tree_n), _ptr(feat_src), _ptr(queries), R, Cc,
            _ptr(nn_pos), _ptr(nn_dist), _ptr(mask)), "kd_query_rows_dev")

    def kd_compact_rows_dev(self, feat_src, coords, R, Cc, tree_pts, tree_col, tree_n,
                            mask=None, built=None):
        self._check(self.L.navgpu_kd_compact_rows_dev(
            self.h, _ptr(feat_src), _ptr(coords), R, Cc, _ptr(tree_pts), _ptr(tree_col),
            _ptr(tree_n), _ptr(mask), _ptr(built)), "kd_compact_rows_dev")

    def kd_query_rows_lazy_dev(self, tree_pts, tree_col, tree_n, feat_src, queries, R, Cc,
                               nn_pos, nn_dist, mask=None, built=None):
        self._check(self.L.navgpu_kd_query_rows_lazy_dev(
            self.h, _ptr(tree_pts), _ptr(tree_col), _ptr(tree_n), _ptr(feat_src),
            _ptr(queries), R, Cc, _ptr(nn_pos), _ptr(nn_dist), _ptr(mask), _ptr(built)),
            "kd_query_rows_lazy_dev")

    def kd_query_rows_lazy_corr_dev(self, tree_pts, tree_col, tree_n, feat_src, queries, R, Cc,
                                    nn_pos, nn_dist, mask, built, ori, sums):
        self._check(self.L.navgpu_kd_query_rows_lazy_corr_dev(
            self.h, _ptr(tree_pts), _ptr(tree_col), _ptr(tree_n), _ptr(feat_src),
            _ptr(queries), R, Cc, _ptr(nn_pos), _ptr(nn_dist), _ptr(mask), _ptr(built),
            _ptr(ori), _ptr(sums)), "kd_query_rows_lazy_corr_dev")

    def rows_corr_dev(self, tree_pts, tree_n, nn_pos, nn_dist, ori, R, Cc, keep, sums):
        self._check(self.L.navgpu_rows_corr_dev(
            self.h, _ptr(tree_pts), _ptr(tree_n), _ptr(nn_pos), _ptr(nn_dist), _ptr(ori),
            R, Cc, _ptr(keep), _ptr(sums)), "rows_corr")

    def rows_corr_list_dev(self, tree_pts, tree_n, nn_pos, nn_dist, ori, R, Cc, lst, count):
        self._check(self.L.navgpu_rows_corr_list_dev(
            self.h, _ptr(tree_pts), _ptr(tree_n), _ptr(nn_pos), _ptr(nn_dist), _ptr(ori), R, Cc,
            _ptr(lst), _ptr(count)), "rows_corr_list_dev")

    def rows_match_dev(self, src, tgt, R, Cc, src_mask, tgt_mask, nn_idx, nn_dist):
        self._check(self.L.navgpu_rows_match_dev(
            self.h, _ptr(src), _ptr(tgt), R, Cc, _ptr(src_mask), _ptr(tgt_mask),
            _ptr(nn_idx), _ptr(nn_dist)), "rows_match_dev")

    def rows_match_batch_dev(self, src, tgt, npairs, R, Cc, src_mask, tgt_mask, nn_idx,
                             nn_dist):
        self._check(self.L.navgpu_rows_match_batch_dev(
            self.h, _ptr(src), _ptr(tgt), npairs, R, Cc, _ptr(src_mask), _ptr(tgt_mask),
            _ptr(nn_idx), _ptr(nn_dist)), "rows_match_batch_dev")

    def knn_dev(self, tgt, nt, queries, nq, k, idx, dist):
        self._check(self.L.navgpu_knn_dev(self.h, _ptr(tgt), nt, _ptr(queries), nq, k,
                                          _ptr(idx), _ptr(dist)), "knn_dev")

    def pair_knn_dev(self, src, tgt, R, Cc, k, src_mask, tgt_mask, idx, dist):
        self._check(self.L.navgpu_pair_knn_dev(
            self.h, _ptr(src), _ptr(tgt), R, Cc, k, _ptr(src_mask), _ptr(tgt_mask),
            _ptr(idx), _ptr(dist)), "pair_knn_dev")
