"""ctypes view of the drop-in C ABI (include/slam.h, kdtree.h, pointcloud.h)
of a libnavslam_<R>x<C>.so: the reference's own structs and entry points
(headers/slam.h:10-28, utils/kdtree.h:7-30, utils/pointcloud.h:32-57), plus
the shim's two extra exports (navslam_context, navslam_last_frame_stats).
Used by bench.py's K5 stream and by the shim tests."""
import ctypes as C
import os

LIBDIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib")
SLAM_MAP_FRAMES = 100  # globalPointCloud[100], headers/slam.h:12


class Point(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double)]


class Pos(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("x", "y", "z", "roll", "pitch", "yaw")]

    @classmethod
    def of(cls, v):
        return cls(*[float(x) for x in v])

    def tolist(self):
        return [self.x, self.y, self.z, self.roll, self.pitch, self.yaw]


class KDNode(C.Structure):
    pass


KDNode._fields_ = [("point", Point), ("left", C.POINTER(KDNode)), ("right", C.POINTER(KDNode))]


def preorder(node):
    out, stack = [], [node]
    while stack:
        n = stack.pop()
        if not n:
            continue
        p = n.contents.point
        out.append((p.x, p.y, p.z))
        stack.append(n.contents.right)
        stack.append(n.contents.left)
    return out


def make_types(R, Cc, frames=SLAM_MAP_FRAMES):
    class PointCloud(C.Structure):
        _fields_ = [("ts", C.c_int), ("pos", Point * Cc * R)]

    class SLAMAttr(C.Structure):
        _fields_ = [("globalPointCloud", PointCloud * frames), ("frameCount", C.c_int),
                    ("kdtree_lastframe", C.POINTER(KDNode) * R), ("error", C.c_double)]
    return PointCloud, SLAMAttr


class Shim:
    """libnavslam_<R>x<C>.so with argtypes set; `cloud()` packs a [R, C, 3]
    float64 array into a PointCloud."""

    def __init__(self, R, Cc):
        self.R, self.C = R, Cc
        # NAVSLAM_LIBDIR: another build of the shim + libnavgpu (A/B runs only)
        self.path = os.path.join(os.environ.get("NAVSLAM_LIBDIR") or LIBDIR,
                                 f"libnavslam_{R}x{Cc}.so")
        from navslam.gpu import load_library
        load_library()  # libnavgpu bound to the process's (torch's) HIP runtime
        L = self.L = C.CDLL(self.path)
        self.PointCloud, self.SLAMAttr = make_types(R, Cc)
        PC, SA = self.PointCloud, self.SLAMAttr
        L.init_slam.argtypes = [C.POINTER(SA), Pos, C.POINTER(PC)]
        L.slam_localization.argtypes = [C.POINTER(SA), C.POINTER(PC), Pos, Pos]
        L.slam_localization.restype = Pos
        L.slam_mapping.argtypes = [C.POINTER(SA), Pos, C.POINTER(PC)]
        L.buildKDTree.restype = C.POINTER(KDNode)
        L.buildKDTree.argtypes = [C.POINTER(Point), C.c_size_t, C.c_int]
        L.freeKDTree.argtypes = [C.POINTER(KDNode)]
        L.nearestNeighborSearch.argtypes = [C.POINTER(KDNode), C.POINTER(Point),
                                            C.POINTER(Point), C.POINTER(C.c_double), C.c_int]
        L.printKDTree.argtypes = [C.POINTER(KDNode), C.c_int]
        L.convertToPointCloud.argtypes = [C.c_void_p, C.c_void_p]
        L.extract_feature.argtypes = [C.POINTER(PC), C.c_void_p]
        L.navslam_context.restype = C.c_void_p
        L.navslam_context.argtypes = []
        L.navslam_last_frame_stats.restype = C.c_int
        L.navslam_last_frame_stats.argtypes = [C.POINTER(C.c_int), C.POINTER(C.c_int),
                                               C.POINTER(C.c_int)]

    def cloud(self, pts, ts=0):
        import numpy as np
        pc = self.PointCloud()
        pc.ts = ts
        a = np.ascontiguousarray(pts, np.float64)
        C.memmove(C.addressof(pc.pos), a.ctypes.data, a.nbytes)
        return pc

    def context(self):
        """The shim's navgpu_ctx* (for navgpu_timing / timing_read)."""
        return self.L.navslam_context()

    def last_frame_stats(self):
        """(feature queries, correspondences after dedup, Adam iterations) of
        the last slam_localization call."""
        q, cp, it = C.c_int(), C.c_int(), C.c_int()
        self.L.navslam_last_frame_stats(C.byref(q), C.byref(cp), C.byref(it))
        return q.value, cp.value, it.value
