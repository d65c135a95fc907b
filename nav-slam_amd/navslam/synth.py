"""Seeded synthetic inputs for the scan-matching path.

No dataset ships with the reference (`dataset/` is gitignored,
/root/reference/.gitignore:2), so every workload is generated here:

* ``l9_pair``  — "L9-shaped" range-image pair: azimuth -180..180 deg over the
  columns, elevation -15..+15 deg over the rows, ray-cast against a fixed room
  with pillars, +U(0,20) mm range noise, 2 % dropouts to (0,0,0) (the
  invalid-point convention of utils/pointcloud.c:24-27). The target is the
  same scene seen from a sensor moved by a known pose step. ``integer_mm``
  rounds coordinates to whole mm, the L9 CSV format
  (visualization/parse_dataset.py:31-33), which makes distance ties real.
* ``uniform_pair`` — K3: x,y,z ~ U[0,1000) mm, arranged as an R x C grid so
  curvature has rows to sweep; source seed 1, target seed 2.
* ``l5_stream`` — 8x8 integer depth grids + IMU poses for the
  src/main.c:247-318 loop (x,y,z in metres, angles in degrees).

Arrays are float64 [R, C, 3], row-major: the reference ``Point`` grid.
"""
import numpy as np

_PILLARS = np.array([[2500.0, 1500.0], [-3000.0, 2000.0], [4000.0, -2500.0],
                     [-1500.0, -3500.0], [6000.0, 3500.0], [-6000.0, -1000.0]])
_PILLAR_R = 300.0
_ROOM = (8000.0, 6000.0, -1500.0, 2500.0)  # |x|<=X, |y|<=Y, z in [Z0, Z1]


def _raycast(origin, dirs):
    """Range along unit `dirs` [N,3] from `origin` to the room / pillars."""
    X, Y, Z0, Z1 = _ROOM
    big = np.full(dirs.shape[0], np.inf)
    t = big.copy()
    with np.errstate(divide="ignore", invalid="ignore"):
        for ax, lo, hi in ((0, -X, X), (1, -Y, Y), (2, Z0, Z1)):
            d = dirs[:, ax]
            tl = (lo - origin[ax]) / d
            th = (hi - origin[ax]) / d
            for tt in (tl, th):
                tt = np.where(tt > 1e-9, tt, np.inf)
                t = np.minimum(t, tt)
        # vertical cylinders: |(o + t d)_xy - c|^2 = r^2
        dx, dy = dirs[:, 0], dirs[:, 1]
        a = dx * dx + dy * dy
        for cx, cy in _PILLARS:
            ox, oy = origin[0] - cx, origin[1] - cy
            b = 2 * (ox * dx + oy * dy)
            c = ox * ox + oy * oy - _PILLAR_R ** 2
            disc = b * b - 4 * a * c
            ok = (disc >= 0) & (a > 0)
            sq = np.sqrt(np.where(ok, disc, 0))
            t1 = np.where(ok, (-b - sq) / (2 * a), np.inf)
            t1 = np.where(t1 > 1e-9, t1, np.inf)
            t = np.minimum(t, t1)
    return t


def _scan(R, C, origin, yaw_deg, rng, dropout=0.02, noise_mm=20.0):
    az = np.deg2rad(np.linspace(-180.0, 180.0, C, endpoint=False))
    el = np.deg2rad(np.linspace(-15.0, 15.0, R))
    AZ, EL = np.meshgrid(az, el)                        # [R, C]
    d_s = np.stack([np.cos(EL) * np.cos(AZ), np.cos(EL) * np.sin(AZ), np.sin(EL)], -1)
    yaw = np.deg2rad(yaw_deg)
    cz, sz = np.cos(yaw), np.sin(yaw)
    Rz = np.array([[cz, -sz, 0.0], [sz, cz, 0.0], [0.0, 0.0, 1.0]])
    d_w = d_s.reshape(-1, 3) @ Rz.T                     # sensor -> world
    rng_mm = _raycast(np.asarray(origin, np.float64), d_w).reshape(R, C)
    rng_mm = rng_mm + rng.uniform(0.0, noise_mm, (R, C))
    pts = d_s * rng_mm[..., None]                       # sensor-frame points
    drop = rng.random((R, C)) < dropout
    pts[drop] = 0.0
    return pts


def l9_pair(R=128, C=2048, seed=5, integer_mm=False,
            step=(120.0, -40.0, 5.0), yaw_step_deg=0.8):
    """(src, tgt) float64 [R, C, 3] clouds of one scene from two poses."""
    rng = np.random.default_rng(seed)
    src = _scan(R, C, (0.0, 0.0, 0.0), 0.0, rng)
    tgt = _scan(R, C, step, yaw_step_deg, rng)
    if integer_mm:
        src = np.round(src)
        tgt = np.round(tgt)
    return np.ascontiguousarray(src), np.ascontiguousarray(tgt)


def uniform_pair(R=512, C=2048, seed_src=1, seed_tgt=2, hi=1000.0):
    """K3: two clouds of R*C points, x,y,z ~ U[0, hi) mm."""
    src = np.random.default_rng(seed_src).uniform(0.0, hi, (R, C, 3))
    tgt = np.random.default_rng(seed_tgt).uniform(0.0, hi, (R, C, 3))
    return src, tgt


def l5_stream(rng, frames, R=8, C=8):
    """Integer depth grids [F, R, C] (mm) and IMU poses [F, 6] in the units
    src/main.c:131-190 reads them (x,y,z metres, angles degrees)."""
    imu = np.zeros((frames, 6))
    depth = np.zeros((frames, R, C), np.int32)
    theta = np.deg2rad(-22.5 + np.arange(C) * 45.0 / (C - 1))
    phi = np.deg2rad(-22.5 + np.arange(R) * 45.0 / (R - 1))
    for f in range(frames):
        x = 0.015 * f + rng.normal(0, 0.002)
        y = 0.004 * f + rng.normal(0, 0.002)
        yaw = 0.3 * f + rng.normal(0, 0.05)
        imu[f] = (x, y, 0.0, rng.normal(0, 0.05), rng.normal(0, 0.05), yaw)
        # wall at 2.6 m, a box 0.9 m closer on the left half, a step below
        base = 2600.0 - 1000.0 * x
        d = np.full((R, C), base)
        d[:, : C // 2 - 1] -= 900.0
        d[R // 2 + 1:, C // 2 + 1:] -= 450.0
        d = d / np.cos(theta)[None, :] ** 0.15 / np.cos(phi)[:, None] ** 0.1
        d = d + rng.integers(-4, 5, (R, C))
        depth[f] = np.round(d).astype(np.int32)
    return depth, imu


def l9_stream(R=128, C=2048, frames=8, seed=11, step=(40.0, 15.0, 0.0), yaw_step_deg=0.25,
              integer_mm=False):
    """K5: sensor-frame L9-shaped scans [F, R, C, 3] along a straight walk
    through the room (``step`` mm and ``yaw_step_deg`` per frame), the input
    of the src/main.c:361-431 L9 loop. Ray-casting costs ~0.4 s per
    128x2048 frame, so long streams replay these frames back and forth
    (``l9_stream_index``)."""
    rng = np.random.default_rng(seed)
    out = np.empty((frames, R, C, 3))
    for f in range(frames):
        origin = (step[0] * f, step[1] * f, step[2] * f)
        out[f] = _scan(R, C, origin, yaw_step_deg * f, rng)
    if integer_mm:
        out = np.round(out)
    return out


def l9_stream_index(i, frames):
    """Frame of a ping-pong replay 0, 1, ..., F-1, F-2, ..., 1, 0, 1, ... so a
    long stream keeps moving continuously."""
    if frames <= 1:
        return 0
    p = 2 * (frames - 1)
    j = i % p
    return j if j < frames else p - j
