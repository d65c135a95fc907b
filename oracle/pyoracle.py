"""ctypes binding of oracle/liboracle.so (the CPU restatement, oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline. The product
package (nav-slam_amd/) never imports this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _d(a):
    return a.ctypes.data_as(_dp)


def _i(a):
    return a.ctypes.data_as(_ip)


class Oracle:
    def __init__(self):
        if not os.path.exists(LIB):
            build()
        L = self.L = C.CDLL(LIB)
        L.orc_convert_to_pointcloud.argtypes = [_ip, C.c_int, C.c_int, _dp]
        L.orc_extract_feature.argtypes = [_dp, C.c_int, C.c_int, _ip, C.c_void_p]
        L.orc_rotation_matrix_deg.argtypes = [C.c_double] * 3 + [_dp]
        L.orc_transform_cloud.argtypes = [_dp, C.c_size_t, _dp, _dp, _dp]
        L.orc_kd_build.argtypes = [_dp, _ip, C.c_size_t]
        L.orc_nth_element.argtypes = [_dp, _ip, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int]
        L.orc_kd_nn.argtypes = [_dp, C.c_size_t, _dp, C.POINTER(C.c_long), _dp]
        L.orc_rows_match.argtypes = [_dp, _dp, C.c_int, C.c_int, _ip, _ip, _ip, _dp]
        L.orc_knn_brute.argtypes = [_dp, C.c_size_t, _dp, C.c_size_t, C.c_int, _ip, _dp]
        L.orc_kd_nn_batch.argtypes = [_dp, C.c_size_t, _dp, C.c_size_t,
                                      C.POINTER(C.c_long), _dp]
        L.orc_ref_nn_batch.argtypes = [C.c_void_p, C.c_void_p, _dp, C.c_size_t, _dp, _dp]
        L.orc_knn_grid.argtypes = [_dp, C.c_size_t, _dp, C.c_size_t, C.c_int, _ip, _dp]
        L.orc_ref_nn_batch_mt.argtypes = [C.c_void_p, C.c_void_p, _dp, C.c_size_t, _dp, _dp]
        L.orc_ref_rows_match_mt.restype = C.c_long
        L.orc_ref_rows_match_mt.argtypes = [C.c_void_p] * 3 + [_dp, _dp, _ip, _ip, C.c_int,
                                                               C.c_int, C.c_int, _dp, _dp]
        L.orc_extract_feature_mt.argtypes = [_dp, C.c_int, C.c_int, _ip, C.c_int]
        L.orc_max_threads.restype = C.c_int
        L.orc_rows_dedup.restype = C.c_int
        L.orc_rows_dedup.argtypes = [_dp, C.c_int, C.c_int, C.c_void_p, _dp, _dp, _dp, _dp, _dp,
                                     C.c_void_p]
        L.orc_slam_create.restype = C.c_void_p
        L.orc_slam_create.argtypes = [C.c_int, C.c_int]
        L.orc_slam_destroy.argtypes = [C.c_void_p]
        L.orc_slam_init.argtypes = [C.c_void_p, _dp, _dp]
        L.orc_slam_localization.argtypes = [C.c_void_p, _dp, _dp, _dp, _dp, _ip, _ip]
        L.orc_slam_mapping.argtypes = [C.c_void_p, _dp, _dp]
        L.orc_slam_error.restype = C.c_double
        L.orc_slam_error.argtypes = [C.c_void_p]
        L.orc_slam_frame_count.restype = C.c_int
        L.orc_slam_frame_count.argtypes = [C.c_void_p]
        L.orc_slam_tree.restype = C.c_size_t
        L.orc_slam_tree.argtypes = [C.c_void_p, C.c_int, C.POINTER(_dp), C.POINTER(_ip)]
        L.orc_slam_last_global.restype = _dp
        L.orc_slam_last_global.argtypes = [C.c_void_p]
        for f in ("orc_ekf_init", "orc_ekf_predict", "orc_ekf_modify"):
            getattr(L, f).argtypes = [C.c_void_p, _dp] + ([_dp] if f == "orc_ekf_predict" else [])
        L.orc_ekf_update_R.argtypes = [C.c_void_p, C.c_double]

    # ---- single functions -------------------------------------------------
    def convert(self, depth):
        depth = np.ascontiguousarray(depth, np.int32)
        R, Cc = depth.shape
        out = np.zeros((R, Cc, 3))
        self.L.orc_convert_to_pointcloud(_i(depth), R, Cc, _d(out))
        return out

    def extract_feature(self, pts, want_curv=False):
        pts = np.ascontiguousarray(pts, np.float64)
        R, Cc = pts.shape[:2]
        mask = np.zeros((R, Cc), np.int32)
        curv = np.zeros((R, Cc)) if want_curv else None
        self.L.orc_extract_feature(_d(pts), R, Cc, _i(mask),
                                   curv.ctypes.data if want_curv else None)
        return (mask, curv) if want_curv else mask

    def rotation(self, roll, pitch, yaw):
        Rm = np.zeros(9)
        self.L.orc_rotation_matrix_deg(roll, pitch, yaw, _d(Rm))
        return Rm

    def transform(self, pts, pos6):
        pts = np.ascontiguousarray(pts, np.float64)
        Rm = self.rotation(pos6[3], pos6[4], pos6[5])
        t = np.ascontiguousarray(pos6[:3], np.float64)
        out = np.zeros_like(pts)
        self.L.orc_transform_cloud(_d(pts), pts.size // 3, _d(Rm), _d(t), _d(out))
        return out

    def nth_element(self, key, perm, first, last, nth):
        """utils/kdtree.c:20-52 on keys[perm[first..last]] (axis 0): returns
        the permutation after the reference's Lomuto quickselect."""
        key = np.asarray(key, np.float64)
        ix = np.ascontiguousarray(perm, np.int32).copy()
        p = np.zeros((len(ix), 3))
        p[:, 0] = key[ix]
        self.L.orc_nth_element(_d(p), _i(ix), first, last, nth, 0)
        return ix

    def kd_build(self, pts):
        """Returns (permuted points, permutation of original indices)."""
        p = np.array(pts, np.float64, order="C").reshape(-1, 3)
        ix = np.arange(len(p), dtype=np.int32)
        self.L.orc_kd_build(_d(p), _i(ix), len(p))
        return p, ix

    def kd_nn(self, tree, q):
        tree = np.ascontiguousarray(tree, np.float64).reshape(-1, 3)
        q = np.ascontiguousarray(q, np.float64)
        pos = C.c_long()
        d = np.zeros(1)
        self.L.orc_kd_nn(_d(tree), len(tree), _d(q), C.byref(pos), _d(d))
        return pos.value, d[0]

    def kd_nn_batch(self, tree, qs):
        tree = np.ascontiguousarray(tree, np.float64).reshape(-1, 3)
        qs = np.ascontiguousarray(qs, np.float64).reshape(-1, 3)
        pos = np.zeros(len(qs), np.int64)
        d = np.zeros(len(qs))
        self.L.orc_kd_nn_batch(_d(tree), len(tree), _d(qs), len(qs),
                               pos.ctypes.data_as(C.POINTER(C.c_long)), _d(d))
        return pos, d

    def ref_nn_batch(self, fn_addr, root, qs):
        qs = np.ascontiguousarray(qs, np.float64).reshape(-1, 3)
        pts = np.zeros_like(qs)
        d = np.zeros(len(qs))
        self.L.orc_ref_nn_batch(fn_addr, root, _d(qs), len(qs), _d(pts), _d(d))
        return pts, d

    def rows_match(self, src, tgt):
        src = np.ascontiguousarray(src, np.float64)
        tgt = np.ascontiguousarray(tgt, np.float64)
        R, Cc = src.shape[:2]
        sm = np.zeros((R, Cc), np.int32)
        tm = np.zeros((R, Cc), np.int32)
        idx = np.zeros((R, Cc), np.int32)
        dist = np.zeros((R, Cc))
        self.L.orc_rows_match(_d(src), _d(tgt), R, Cc, _i(sm), _i(tm), _i(idx), _d(dist))
        return sm, tm, idx, dist

    def knn_brute(self, tgt, qs, k):
        tgt = np.ascontiguousarray(tgt, np.float64).reshape(-1, 3)
        qs = np.ascontiguousarray(qs, np.float64).reshape(-1, 3)
        idx = np.zeros((len(qs), k), np.int32)
        dist = np.zeros((len(qs), k))
        self.L.orc_knn_brute(_d(tgt), len(tgt), _d(qs), len(qs), k, _i(idx), _d(dist))
        return idx, dist


    def knn_grid(self, tgt, qs, k):
        """Same result as knn_brute (pinned by tests/test_oracle.py), grid +
        OpenMP: fast enough for every query of the 1M K3 pair."""
        tgt = np.ascontiguousarray(tgt, np.float64).reshape(-1, 3)
        qs = np.ascontiguousarray(qs, np.float64).reshape(-1, 3)
        idx = np.zeros((len(qs), k), np.int32)
        dist = np.zeros((len(qs), k))
        self.L.orc_knn_grid(_d(tgt), len(tgt), _d(qs), len(qs), k, _i(idx), _d(dist))
        return idx, dist

    def ref_nn_batch_mt(self, fn_addr, root, qs):
        qs = np.ascontiguousarray(qs, np.float64).reshape(-1, 3)
        pts = np.zeros_like(qs)
        d = np.zeros(len(qs))
        self.L.orc_ref_nn_batch_mt(fn_addr, root, _d(qs), len(qs), _d(pts), _d(d))
        return pts, d

    def extract_feature_mt(self, pts, threads):
        pts = np.ascontiguousarray(pts, np.float64)
        R, Cc = pts.shape[:2]
        mask = np.zeros((R, Cc), np.int32)
        self.L.orc_extract_feature_mt(_d(pts), R, Cc, _i(mask), threads)
        return mask

    def ref_rows_match(self, fns, src, tgt, smask, tmask, threads):
        """Per-row build + 1-NN through the reference's own functions
        fns = (buildKDTree, nearestNeighborSearch, freeKDTree) addresses.
        Returns (nearest points [R,C,3], distances [R,C] (+inf where no
        query), number of queries)."""
        src = np.ascontiguousarray(src, np.float64)
        tgt = np.ascontiguousarray(tgt, np.float64)
        R, Cc = src.shape[:2]
        pts = np.zeros_like(src)
        d = np.full((R, Cc), np.inf)
        sm = np.ascontiguousarray(smask, np.int32)
        tm = np.ascontiguousarray(tmask, np.int32)
        n = self.L.orc_ref_rows_match_mt(fns[0], fns[1], fns[2], _d(src), _d(tgt), _i(sm),
                                         _i(tm), R, Cc, threads, _d(pts), _d(d))
        return pts, d, int(n)

    def rows_dedup(self, trees, pos, dist, ori):
        """src/slam.c:236-284 over per-row trees [R,C,3] and per-cell 1-NN
        results pos/dist [R,C]: (ori [n,3], near [n,3], dist [n], grid index
        [n]) in the reference list's order."""
        trees = np.ascontiguousarray(trees, np.float64)
        R, Cc = trees.shape[:2]
        pos = np.ascontiguousarray(pos, np.int64)
        dist = np.ascontiguousarray(dist, np.float64)
        ori = np.ascontiguousarray(ori, np.float64)
        N = R * Cc
        o, nr, d, g = np.zeros((N, 3)), np.zeros((N, 3)), np.zeros(N), np.zeros(N, np.int64)
        n = self.L.orc_rows_dedup(_d(trees), R, Cc, pos.ctypes.data, _d(dist), _d(ori), _d(o),
                                  _d(nr), _d(d), g.ctypes.data)
        return o[:n], nr[:n], d[:n], g[:n]

    def max_threads(self):
        return int(self.L.orc_max_threads())


class OracleSlam:
    """src/slam.c:134-431 frame loop at runtime dims (oracle restatement)."""

    def __init__(self, orc, R, Cc):
        self.o, self.R, self.C = orc, R, Cc
        self.h = orc.L.orc_slam_create(R, Cc)

    def __del__(self):
        try:
            self.o.L.orc_slam_destroy(self.h)
        except Exception:
            pass

    def init(self, pos6, lidar):
        self.o.L.orc_slam_init(self.h, _d(np.ascontiguousarray(pos6, np.float64)),
                               _d(np.ascontiguousarray(lidar, np.float64)))

    def localization(self, lidar, pred6, last6):
        out = np.zeros(6)
        it = np.zeros(1, np.int32)
        nc = np.zeros(1, np.int32)
        self.o.L.orc_slam_localization(self.h, _d(np.ascontiguousarray(lidar, np.float64)),
                                       _d(np.ascontiguousarray(pred6, np.float64)),
                                       _d(np.ascontiguousarray(last6, np.float64)),
                                       _d(out), _i(it), _i(nc))
        return out, int(it[0]), int(nc[0])

    def mapping(self, pos6, lidar):
        self.o.L.orc_slam_mapping(self.h, _d(np.ascontiguousarray(pos6, np.float64)),
                                  _d(np.ascontiguousarray(lidar, np.float64)))

    @property
    def error(self):
        return self.o.L.orc_slam_error(self.h)

    @property
    def frame_count(self):
        return self.o.L.orc_slam_frame_count(self.h)

    def tree(self, r):
        p = _dp()
        c = _ip()
        n = self.o.L.orc_slam_tree(self.h, r, C.byref(p), C.byref(c))
        pts = np.ctypeslib.as_array(p, (max(n, 1) * 3,))[: 3 * n].reshape(-1, 3).copy()
        cols = np.ctypeslib.as_array(c, (max(n, 1),))[:n].copy()
        return pts, cols

    def last_global(self):
        g = self.o.L.orc_slam_last_global(self.h)
        return np.ctypeslib.as_array(g, (self.R * self.C * 3,)).reshape(self.R, self.C, 3).copy()


class OracleEkf:
    def __init__(self, orc, pos6):
        self.o = orc
        self.buf = np.zeros(6 + 3 * 36)
        orc.L.orc_ekf_init(self.buf.ctypes.data, _d(np.ascontiguousarray(pos6, np.float64)))

    def predict(self, last6, cur6):
        self.o.L.orc_ekf_predict(self.buf.ctypes.data, _d(np.asarray(last6, np.float64)),
                                 _d(np.asarray(cur6, np.float64)))

    def modify(self, meas6):
        self.o.L.orc_ekf_modify(self.buf.ctypes.data, _d(np.asarray(meas6, np.float64)))

    def update_R(self, err):
        self.o.L.orc_ekf_update_R(self.buf.ctypes.data, float(err))

    @property
    def pos(self):
        return self.buf[:6].copy()
