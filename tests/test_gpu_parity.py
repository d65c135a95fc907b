"""HIP path vs the oracle restatement and the reference's golden fixtures.

Every comparison is bit-exact (masks, permutations, indices, fp64 distances
and poses): integer/index work must be, and the fp64 arithmetic is kept in
the reference's operation order (-ffp-contract=off), so the tolerance the
north star allows (1e-5 relative on distances/curvature) is not needed —
tests assert equality and report the worst relative error if it ever breaks.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from navslam.gpu import NavGpu
    g = NavGpu(0)
    yield g
    g.close()


# every K3 query pass the library can select (NAVGPU_KNN_MODE): 1 k_knnw,
# 2 k_knng on the row neighbourhood lists
KNN_MODES = (1, 2)


def _knn_ctx(mode, **env):
    import os
    from navslam.gpu import NavGpu
    env = dict(env, NAVGPU_KNN_MODE=str(mode))
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return NavGpu(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module", params=KNN_MODES, ids=lambda m: f"mode{m}")
def kgpu(request):
    g = _knn_ctx(request.param)
    yield g
    g.close()


_ORC_MEMO = {}


def _memo(key, fn):
    """oracle answers shared by the parametrised query passes"""
    if key not in _ORC_MEMO:
        _ORC_MEMO[key] = fn()
    return _ORC_MEMO[key]


def _eq(a, b, msg=""):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f":
        same = (a == b) | (np.isnan(a) & np.isnan(b))
        if not same.all():
            with np.errstate(all="ignore"):
                rel = np.nanmax(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))
            raise AssertionError(f"{msg}: {(~same).sum()} mismatches, max rel {rel:.3e}")
    else:
        np.testing.assert_array_equal(a, b, err_msg=msg)


# ------------------------------------------------------------------ R1 / R2
def test_curvature_matches_reference_golden(gpu, golden):
    g = golden("curv8x8")
    pts = g["pts"].reshape(-1, 8, 3)          # stack the 8x8 clouds as rows
    mask = gpu.curvature(pts)
    _eq(mask.reshape(-1, 8, 8), g["mask"], "curv8x8 masks")


def test_curvature_values_bit_exact(gpu, orc):
    rng = np.random.default_rng(3)
    clouds = [rng.uniform(-5000, 5000, (64, 301, 3)),
              np.round(rng.uniform(-3000, 3000, (32, 257, 3))),
              rng.normal(0, 1, (16, 129, 3)) * 10.0 ** rng.integers(-30, 30, (16, 129, 1)),
              np.zeros((4, 64, 3))]
    c = rng.uniform(0, 10, (8, 97, 3))
    c[:, 0:96:3] = c[:, 1:97:3]               # duplicate neighbours
    clouds.append(c)
    for pts in clouds:
        m_ref, c_ref = orc.extract_feature(pts, want_curv=True)
        m, cv = gpu.curvature(pts, want_curv=True)
        _eq(m, m_ref, "mask")
        _eq(cv, c_ref, "curvature")


def test_project_matches_reference_golden(gpu, golden, orc):
    g = golden("convert8x8")
    for d, p in zip(g["depth"], g["pts"]):
        _eq(gpu.project(d), p, "convertToPointCloud")
    rng = np.random.default_rng(4)
    d = rng.integers(-200, 9000, (64, 512)).astype(np.int32)
    _eq(gpu.project(d), orc.convert(d), "64x512 projection")


# ------------------------------------------------------------------ R5 build
def _golden_sets(g):
    off = qoff = 0
    for n, nq in zip(g["n"], g["nq"]):
        yield (g["pts"][off:off + n], g["perm"][off:off + n], g["q"][qoff:qoff + nq],
               g["nn"][qoff:qoff + nq], g["nnd"][qoff:qoff + nq])
        off += n
        qoff += nq


def test_kd_build_permutation_matches_reference(gpu, golden):
    for pts, perm, *_ in _golden_sets(golden("kdtree")):
        _eq(gpu.kd_build(pts), perm, f"buildKDTree n={len(pts)}")


@pytest.mark.parametrize("n,depth0", [(3000, 0), (5000, 1), (70000, 0), (9, 2)])
def test_kd_build_large_and_depth_offset(gpu, orc, n, depth0):
    rng = np.random.default_rng(n + depth0)
    pts = np.round(rng.uniform(0, 40, (n, 3)))       # heavy duplicates
    ref = pts.copy()
    ix = np.arange(n, dtype=np.int32)
    # oracle with a shifted root axis: rotate coordinates so axis (d0+l)%3
    # becomes l%3, build, rotate back
    rot = np.roll(ref, -depth0, axis=1)
    t, _ = orc.kd_build(rot)
    _eq(gpu.kd_build(pts, depth0), np.roll(t, depth0, axis=1), f"n={n} depth0={depth0}")
    del ix


@pytest.mark.parametrize("n,depth0,integer", [(1_000_000, 0, False), (1_000_000, 2, True),
                                              (300_001, 1, False)])
def test_kd_build_million_level_parallel(gpu, orc, n, depth0, integer):
    """buildKDTree (utils/kdtree.c:20-82) beyond one workgroup's LDS: the
    level-parallel build (a workgroup per subarray per level, then one per
    LDS-sized subtree) gives the reference permutation, also with heavy
    duplicates and a shifted root axis."""
    rng = np.random.default_rng(n + depth0)
    pts = rng.uniform(-5000, 5000, (n, 3))
    if integer:
        pts = np.round(pts / 50.0)
    rot = np.roll(pts, -depth0, axis=1)
    t, _ = orc.kd_build(rot)
    _eq(gpu.kd_build(pts, depth0), np.roll(t, depth0, axis=1), f"n={n} depth0={depth0}")


def test_kd_build_adversarial_orders(gpu, orc):
    """Inputs on which Lomuto's last-element pivot degenerates: a tree-ordered
    array (the output of a previous build) and an x-sorted one. These give
    the grid-wide passes long tape chains (the jump rounds and the scatter's
    own chain following) and hundreds of quickselect steps per level."""
    rng = np.random.default_rng(31)
    pts = rng.uniform(0, 1000, (150_000, 3))
    tree, _ = orc.kd_build(pts)
    t2, _ = orc.kd_build(tree.copy())
    _eq(gpu.kd_build(tree), t2, "tree-ordered input")
    s = rng.uniform(0, 1000, (20_000, 3))
    s = s[np.argsort(s[:, 0], kind="stable")]
    ts, _ = orc.kd_build(s.copy())
    _eq(gpu.kd_build(s), ts, "x-sorted input")


@pytest.mark.parametrize("n", [3000, 100_000])
def test_kd_build_nonfinite_and_signed_zeros(gpu, orc, n):
    """buildKDTree's Lomuto compares (utils/kdtree.c:20-45) on NaN, +-inf and
    -0.0 / +0.0 coordinates, in one workgroup's LDS (3000) and through the
    grid-wide passes (100k). Compared bit for bit (uint64 view), so a -0.0
    landing where the reference puts a +0.0 is caught."""
    rng = np.random.default_rng(n + 7)
    pts = np.round(rng.uniform(-20, 20, (n, 3)))
    m = n // 50
    for v in (np.nan, np.inf, -np.inf, -0.0, 0.0):
        pts[rng.integers(0, n, m), rng.integers(0, 3, m)] = v
    t, _ = orc.kd_build(pts.copy())
    got = gpu.kd_build(pts)
    np.testing.assert_array_equal(np.asarray(got).view(np.uint64), t.view(np.uint64),
                                  err_msg=f"n={n}")


def test_kd_build_level_parallel_equals_single_workgroup(gpu, monkeypatch):
    rng = np.random.default_rng(9)
    pts = np.round(rng.uniform(0, 300, (40000, 3)))
    a = gpu.kd_build(pts, 1)
    monkeypatch.setenv("NAVGPU_KD_ONE_WG", "1")
    b = gpu.kd_build(pts, 1)
    _eq(a, b, "level-parallel vs single-workgroup build")



@pytest.mark.parametrize("kind", ["random", "scanlike", "duplicates", "nonfinite"])
def test_nth_element_matches_reference(gpu, orc, kind):
    """The per-row builds' nth_element (one wave: ordinary passes over
    64-position chunks and the register-resident pass; the 1024-thread block
    pass with its hand-over to wave 0) against the oracle's
    utils/kdtree.c:20-52 on windows of 2..4000 positions at any offset,
    scan-like keys (long left-descent chains) and non-finite keys included."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(len(kind) + 40)
    for trial in range(40):
        n = int(rng.integers(2, 4000)) if trial % 3 else int(rng.integers(2, 300))
        if kind == "scanlike":
            key = np.cumsum(rng.normal(-0.3, 1.0, n))
        elif kind == "duplicates":
            key = np.round(rng.uniform(0, 6, n))
        else:
            key = rng.uniform(-1, 1, n)
        if kind == "nonfinite":
            for v in (np.inf, -np.inf, np.nan, 0.0, -0.0):
                key[rng.integers(0, n, 3)] = v
        perm = rng.permutation(n).astype(np.int32)
        first = int(rng.integers(0, n))
        last = int(rng.integers(first, n))
        nth = int(rng.integers(first, last + 1))
        ref = orc.nth_element(key, perm, first, last, nth)
        for block in (False, True):
            kd = torch.tensor(key, dtype=torch.float64, device=dev)
            pd = torch.tensor(perm, dtype=torch.int32, device=dev)
            gpu.debug_nth_element(kd, pd, first, last, nth, block=block)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(pd.cpu().numpy(), ref,
                                          err_msg=f"{kind} n={n} [{first},{last}] nth={nth} "
                                                  f"block={block}")


# ------------------------------------------------------ R4-R6 per-row mode
def test_rows_match_l9_golden(gpu, golden):
    g = golden("rows_l9")
    for tag in ("f", "i"):
        src, tgt = g[f"src_{tag}"], g[f"tgt_{tag}"]
        sm, tm, idx, dist = gpu.rows_match(src, tgt)
        _eq(sm, g[f"smask_{tag}"], "src mask")
        _eq(tm, g[f"tmask_{tag}"], "tgt mask")
        q = sm == 1
        _eq(dist[q], g[f"nnd_{tag}"][q], "distances")
        hit = q & (idx >= 0)
        _eq(tgt.reshape(-1, 3)[idx[hit]], g[f"nn_{tag}"][hit], "nearest points")


@pytest.mark.parametrize("integer", [False, True])
def test_rows_match_k2_shape_vs_oracle(gpu, orc, integer):
    from navslam.synth import l9_pair
    src, tgt = l9_pair(128, 2048, seed=11, integer_mm=integer)
    ref = orc.rows_match(src, tgt)
    got = gpu.rows_match(src, tgt)
    for a, b, name in zip(got, ref, ("src_mask", "tgt_mask", "nn_idx", "nn_dist")):
        _eq(a, b, name)
    assert (ref[2] >= 0).sum() > 100000


def test_rows_match_batch_equals_per_pair(gpu, orc):
    """K4 batch launch over [pair][R][C] == one rows_match per pair (indices
    relative to each pair), and the oracle."""
    import torch
    from navslam.synth import l9_pair
    R, Cc, P = 16, 512, 3
    pairs = [l9_pair(R, Cc, seed=40 + p, integer_mm=p == 1) for p in range(P)]
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(np.stack([a for a, _ in pairs])).to(dev)
    tgt = torch.from_numpy(np.stack([b for _, b in pairs])).to(dev)
    i32 = lambda: torch.full((P, R, Cc), -7, dtype=torch.int32, device=dev)  # noqa: E731
    sm, tm, idx = i32(), i32(), i32()
    dist = torch.zeros((P, R, Cc), dtype=torch.float64, device=dev)
    gpu.rows_match_batch_dev(src, tgt, P, R, Cc, sm, tm, idx, dist)
    torch.cuda.synchronize()
    for p, (a, b) in enumerate(pairs):
        ref = orc.rows_match(a, b)
        got = (sm[p].cpu().numpy(), tm[p].cpu().numpy(), idx[p].cpu().numpy(),
               dist[p].cpu().numpy())
        for x, y, name in zip(got, ref, ("src_mask", "tgt_mask", "nn_idx", "nn_dist")):
            _eq(x, y, f"pair {p} {name}")


def test_rows_match_batch_k4_full_size(gpu, orc):
    """K4 at full size, as bench.py --workload k4 builds it: 256 pairs of
    128 x 2048 (8 distinct L9-shaped pairs, seeds 5..12, cycled; here pair 3
    of every 8 is integer-mm, L9's native format) in ONE batch launch of
    rows_match_batch_dev, every pair compared with the single-pair rows_match
    of the same clouds, and each of the 8 distinct single-pair results
    compared with the oracle's rows_match (pinned to the reference by
    test_oracle.py and the K2 digests)."""
    import torch
    from navslam.synth import l9_pair
    R, Cc, P, ND = 128, 2048, 256, 8
    distinct = [l9_pair(R, Cc, seed=p + 5, integer_mm=p == 3) for p in range(ND)]
    dev = torch.device("cuda", 0)
    src = torch.stack([torch.from_numpy(distinct[p % ND][0]) for p in range(P)]).to(dev)
    tgt = torch.stack([torch.from_numpy(distinct[p % ND][1]) for p in range(P)]).to(dev)
    i32 = lambda: torch.full((P, R, Cc), -7, dtype=torch.int32, device=dev)  # noqa: E731
    sm, tm, idx = i32(), i32(), i32()
    dist = torch.zeros((P, R, Cc), dtype=torch.float64, device=dev)
    gpu.rows_match_batch_dev(src, tgt, P, R, Cc, sm, tm, idx, dist)
    torch.cuda.synchronize()
    del src, tgt
    singles = [gpu.rows_match(a, b) for a, b in distinct]
    assert (singles[3][2] >= 0).sum() > 100000  # the integer-mm pair has work
    names = ("src_mask", "tgt_mask", "nn_idx", "nn_dist")
    for d, (a, b) in enumerate(distinct):  # every distinct pair pinned to the oracle
        for x, y, name in zip(singles[d], orc.rows_match(a, b), names):
            _eq(x, y, f"distinct pair {d} (seed {d + 5}) {name} vs oracle")
    got_all = [t.cpu().numpy() for t in (sm, tm, idx, dist)]
    for p in range(P):
        for x, y, name in zip(got_all, singles[p % ND], names):
            _eq(x[p], y, f"pair {p} {name}")


def test_rows_match_batch_lean_path(gpu, orc, monkeypatch):
    """A batch of >= 1024 rows takes the lean two-rows-per-CU kernel
    (k_rows_match_lean): same masks, indices and distances as the oracle and
    as the resident kernel (NAVGPU_ROWS_NO_LEAN=1)."""
    import torch
    from navslam.synth import l9_pair
    R, Cc, P = 64, 300, 16
    pairs = [l9_pair(R, Cc, seed=60 + p, integer_mm=p % 3 == 1) for p in range(P)]
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(np.stack([a for a, _ in pairs])).to(dev)
    tgt = torch.from_numpy(np.stack([b for _, b in pairs])).to(dev)

    def run():
        i32 = lambda: torch.full((P, R, Cc), -7, dtype=torch.int32, device=dev)  # noqa: E731
        sm, tm, idx = i32(), i32(), i32()
        dist = torch.zeros((P, R, Cc), dtype=torch.float64, device=dev)
        gpu.rows_match_batch_dev(src, tgt, P, R, Cc, sm, tm, idx, dist)
        torch.cuda.synchronize()
        return [t.cpu().numpy() for t in (sm, tm, idx, dist)]
    lean = run()
    monkeypatch.setenv("NAVGPU_ROWS_NO_LEAN", "1")
    resident = run()
    names = ("src_mask", "tgt_mask", "nn_idx", "nn_dist")
    for x, y, name in zip(lean, resident, names):
        _eq(x, y, f"lean vs resident {name}")
    for p in (0, 1, P - 1):
        ref = orc.rows_match(*pairs[p])
        for x, y, name in zip(lean, ref, names):
            _eq(x[p], y, f"pair {p} {name}")


def test_rows_match_dev_without_masks(gpu, orc):
    """navgpu_rows_match_dev with NULL masks (the screen then keeps its masks
    in the context's workspace), odd widths (C not a multiple of the 32-point
    screen chunk, single-split and multi-split launches): the same matches as
    the oracle."""
    import torch
    from navslam.synth import l9_pair
    dev = torch.device("cuda", 0)
    for R, Cc, seed in ((7, 37, 1), (40, 1000, 2), (130, 777, 3)):
        a, b = l9_pair(R, Cc, seed=seed, integer_mm=seed == 2)
        src, tgt = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
        idx = torch.full((R, Cc), -7, dtype=torch.int32, device=dev)
        dist = torch.zeros((R, Cc), dtype=torch.float64, device=dev)
        rc = gpu.L.navgpu_rows_match_dev(gpu.h, C.c_void_p(src.data_ptr()),
                                         C.c_void_p(tgt.data_ptr()), R, Cc, None, None,
                                         C.c_void_p(idx.data_ptr()), C.c_void_p(dist.data_ptr()))
        assert rc == 0
        torch.cuda.synchronize()
        ref = orc.rows_match(a, b)
        _eq(idx.cpu().numpy(), ref[2], f"{R}x{Cc} nn_idx")
        _eq(dist.cpu().numpy(), ref[3], f"{R}x{Cc} nn_dist")


def test_rows_match_edge_cases(gpu, orc):
    rng = np.random.default_rng(5)
    cases = [np.zeros((3, 5, 3)),                                   # C < 5: no window
             rng.uniform(0, 10, (2, 4, 3)),
             np.round(rng.uniform(0, 3, (16, 64, 3))),             # massive ties
             np.tile(rng.uniform(0, 1, (1, 1, 3)), (4, 33, 1))]   # identical points
    big = rng.uniform(-1e4, 1e4, (2, 2304, 3))                    # widest rows
    cases.append(big)
    for c in cases:
        t = c[::-1].copy() + 0.5 * (c.shape[1] % 2)
        _eq(np.stack(gpu.rows_match(c, t)[2:3]), np.stack(orc.rows_match(c, t)[2:3]),
            f"shape {c.shape}")
        _eq(gpu.rows_match(c, t)[3], orc.rows_match(c, t)[3], f"dist {c.shape}")


def test_rows_match_nonfinite_and_dense_features(gpu, orc):
    """Per-row mode on inputs the L9 generator never makes: non-finite
    coordinates (NaN / +-inf never pass the curvature test and never win a
    distance comparison in the reference; utils/kdtree.c:117, src/slam.c:11-61)
    and zig-zag rows where almost every point is a feature (the widest trees
    and the longest Lomuto chains per row)."""
    from navslam.synth import l9_pair
    rng = np.random.default_rng(31)
    src, tgt = l9_pair(32, 512, seed=4)
    for a in (src, tgt):
        for v in (np.nan, np.inf, -np.inf):
            r, c, ax = rng.integers(0, 32, 60), rng.integers(0, 512, 60), rng.integers(0, 3, 60)
            a[r, c, ax] = v
    zz = np.zeros((8, 1024, 3))
    zz[..., 0] = np.arange(1024)[None, :] * 10.0
    zz[..., 1] = np.where(np.arange(1024) % 2, 50.0, -50.0)[None, :] + rng.normal(0, 1, (8, 1024))
    zz[..., 2] = np.arange(8)[:, None] * 100.0
    for s_, t_, name in ((src, tgt, "non-finite"), (zz, zz[:, ::-1].copy() + 3.0, "zig-zag")):
        got = gpu.rows_match(s_, t_)
        ref = orc.rows_match(s_, t_)
        for a, b, what in zip(got, ref, ("src_mask", "tgt_mask", "nn_idx", "nn_dist")):
            _eq(a, b, f"{name}: {what}")


@pytest.mark.parametrize("f32", ["1", "0"])
def test_rows_screen_vs_tree_path(gpu, orc, monkeypatch, f32):
    """The screened per-row path (exact argmin, the reference tree only for
    rows with a tie) == the tree on every row (NAVGPU_ROWS_SCREEN=0) == the
    oracle, on data that stresses the screen's argument: integer ties,
    non-finite coordinates, distances whose squares underflow, duplicate
    points, large offsets (utils/kdtree.c:110-152); with the f32 pre-screen
    (k_rows_screen32, NAVGPU_SCREEN_F32=1: its certificate must fall back to
    the f64 scan on near-ties a few ulps apart, coordinates beyond the f32
    range and rows whose first feature is far from the rest) and without."""
    monkeypatch.setenv("NAVGPU_SCREEN_F32", f32)
    from navslam.synth import l9_pair
    rng = np.random.default_rng(77)
    cases = []
    src, tgt = l9_pair(32, 512, seed=5)
    cases.append(("l9 f64", src, tgt))
    cases.append(("l9 integer", *l9_pair(32, 512, seed=6, integer_mm=True)))
    s2, t2 = src.copy(), tgt.copy()
    s2[3, 100:140, 1] = np.nan
    t2[4, 200:260, 0] = np.inf
    t2[5, 10:400:7, 2] = np.nan
    s2[6, 300:340] = -np.inf
    cases.append(("non-finite", s2, t2))
    tiny = rng.uniform(0, 1, (4, 256, 3)) * 1e-160
    cases.append(("tiny", tiny, tiny[:, ::-1].copy() * 1.0000001))
    dup = np.round(rng.uniform(0, 50, (8, 300, 3)))
    cases.append(("duplicates", dup, dup[::-1].copy()))
    off = rng.uniform(0, 100, (8, 700, 3)) + 1e9
    cases.append(("offset", off, off + rng.uniform(-1, 1, off.shape)))
    huge = rng.uniform(-1, 1, (4, 300, 3)) * np.array([1e20, 1e39, 1e300, 1e20])[:, None, None]
    cases.append(("huge", huge, huge[:, ::-1].copy() * 0.999))
    # near-ties: every target has a partner mirrored about the query grid
    # plane, nudged by a few ulps (the f32 keys cannot tell them apart)
    base = rng.uniform(-20, 20, (8, 256, 3))
    mir = base.copy()
    mir[..., 0] = -mir[..., 0]
    mir = np.nextafter(mir, np.inf)
    near_t = np.concatenate([base, mir], axis=1)
    near_s = np.zeros_like(near_t)
    near_s[..., 1:] = near_t[..., 1:] + rng.uniform(-0.5, 0.5, near_t[..., 1:].shape)
    cases.append(("near-ties", near_s, near_t))
    names = ("src_mask", "tgt_mask", "nn_idx", "nn_dist")
    for label, s, t in cases:
        monkeypatch.delenv("NAVGPU_ROWS_SCREEN", raising=False)
        got = gpu.rows_match(s, t)
        monkeypatch.setenv("NAVGPU_ROWS_SCREEN", "0")
        tree = gpu.rows_match(s, t)
        ref = orc.rows_match(s, t)
        for a, b, c, name in zip(got, tree, ref, names):
            _eq(a, b, f"{label}: screen vs tree {name}")
            _eq(a, c, f"{label}: screen vs oracle {name}")


@pytest.mark.parametrize("query_tree", ["0", "1"])
def test_split_build_query_vs_oracle(gpu, orc, monkeypatch, query_tree):
    """kd_build_rows_dev + kd_query_rows_dev on device tensors (slam.c split:
    features from the lidar frame, coordinates from a transformed frame).
    The query returns the reference's Point: its position, or for
    bit-identical duplicates a position holding the same coordinates; both
    the screen (default) and the tree walk (NAVGPU_ROWS_QUERY_TREE=1)."""
    monkeypatch.setenv("NAVGPU_ROWS_QUERY_TREE", query_tree)
    import torch
    from navslam.synth import l9_pair
    R, Cc = 64, 1024
    lid, lid2 = l9_pair(R, Cc, seed=21, integer_mm=True)
    Rm = orc.rotation(1.5, -0.7, 12.0)
    coords = np.einsum("ij,rcj->rci", Rm.reshape(3, 3), lid)  # any coordinates
    coords = coords + np.array([100.0, -20.0, 3.0])
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_lid, d_coords, d_lid2 = t(lid), t(coords), t(lid2)
    tree = torch.zeros((R, Cc, 3), dtype=torch.float64, device=dev)
    tcol = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
    tn = torch.zeros(R, dtype=torch.int32, device=dev)
    mask = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
    gpu.kd_build_rows_dev(d_lid, d_coords, R, Cc, tree, tcol, tn, mask)
    pos = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
    dist = torch.zeros((R, Cc), dtype=torch.float64, device=dev)
    qmask = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
    gpu.kd_query_rows_dev(tree, tn, d_lid2, d_lid2, R, Cc, pos, dist, qmask)
    gpu.sync()
    fm = orc.extract_feature(lid)
    _eq(mask.cpu().numpy(), fm, "build mask")
    qm = orc.extract_feature(lid2)
    _eq(qmask.cpu().numpy(), qm, "query mask")
    tree, tn, pos, dist = tree.cpu().numpy(), tn.cpu().numpy(), pos.cpu().numpy(), dist.cpu().numpy()
    tcol = tcol.cpu().numpy()
    for r in range(R):
        cols = np.nonzero(fm[r] == 1)[0]
        rt, rix = orc.kd_build(coords[r, cols])
        assert tn[r] == len(cols)
        _eq(tree[r, :len(cols)], rt, f"row {r} tree")
        _eq(tcol[r, :len(cols)], cols[rix], f"row {r} cols")
        for c in np.nonzero(qm[r] == 1)[0]:
            p, d = orc.kd_nn(rt, lid2[r, c])
            assert (pos[r, c] >= 0) == (p >= 0) and dist[r, c] == d, (r, c)
            if p >= 0:
                assert tree[r, pos[r, c]].tobytes() == rt[p].tobytes(), (r, c)
        assert (pos[r][qm[r] == 0] == -1).all()


@pytest.mark.parametrize("seed,integer_mm,R,Cc", [(5, True, 128, 2048), (5, False, 64, 1024)])
def test_lazy_rows_vs_oracle(gpu, orc, seed, integer_mm, R, Cc):
    """kd_compact_rows_dev + kd_query_rows_lazy_dev (the shim's K5 path with
    NAVSLAM_HOST_TREES=0): a row stays in column order unless one of its
    queries met a distance tie, and then holds the reference's tree (and
    column map) exactly; every query's distance equals the oracle's KD walk
    and its position holds the coordinates of the reference's Point.
    Integer-millimetre ranges at the K2 shape make ties common (K2i: 83 of
    128 rows), so some rows must be rebuilt."""
    import torch
    from navslam.synth import l9_pair
    lid, lid2 = l9_pair(R, Cc, seed=seed, integer_mm=integer_mm)
    if integer_mm:  # the K2i pair as it is: integer coordinates on both sides
        coords = lid.copy()
    else:           # features from one frame, coordinates from a moved one
        Rm = orc.rotation(1.5, -0.7, 12.0)
        coords = np.einsum("ij,rcj->rci", Rm.reshape(3, 3), lid) + np.array([100.0, -20.0, 3.0])
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_lid, d_coords, d_lid2 = t(lid), t(coords), t(lid2)
    tree = torch.zeros((R, Cc, 3), dtype=torch.float64, device=dev)
    tcol = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
    tn = torch.zeros(R, dtype=torch.int32, device=dev)
    mask = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
    pos = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
    dist = torch.zeros((R, Cc), dtype=torch.float64, device=dev)
    qmask = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
    built = torch.full((R,), 7, dtype=torch.int32, device=dev)  # compaction zeroes it
    pos2 = torch.zeros_like(pos)
    dist2 = torch.zeros_like(dist)
    torch.cuda.synchronize()  # (the library runs on its own stream)
    gpu.kd_compact_rows_dev(d_lid, d_coords, R, Cc, tree, tcol, tn, mask, built)
    gpu.kd_query_rows_lazy_dev(tree, tcol, tn, d_lid2, d_lid2, R, Cc, pos, dist, qmask, built)
    gpu.sync()
    # a second lazy query over the same rows: rows the first one
    # rebuilt are walked as they stand, not rebuilt again; same answers
    tree1, tcol1 = tree.clone(), tcol.clone()
    torch.cuda.synchronize()
    gpu.kd_query_rows_lazy_dev(tree, tcol, tn, d_lid2, d_lid2, R, Cc, pos2, dist2, None, built)
    gpu.sync()
    _eq(tree.cpu().numpy(), tree1.cpu().numpy(), "second lazy query: rows unchanged")
    _eq(tcol.cpu().numpy(), tcol1.cpu().numpy(), "second lazy query: columns unchanged")
    _eq(pos2.cpu().numpy(), pos.cpu().numpy(), "second lazy query: positions")
    _eq(dist2.cpu().numpy(), dist.cpu().numpy(), "second lazy query: distances")
    nb = built.cpu().numpy()
    fm = orc.extract_feature(lid)
    _eq(mask.cpu().numpy(), fm, "build mask")
    qm = orc.extract_feature(lid2)
    _eq(qmask.cpu().numpy(), qm, "query mask")
    tree, tn, pos, dist = tree.cpu().numpy(), tn.cpu().numpy(), pos.cpu().numpy(), dist.cpu().numpy()
    tcol = tcol.cpu().numpy()
    rebuilt = 0
    for r in range(R):
        cols = np.nonzero(fm[r] == 1)[0]
        n = len(cols)
        assert tn[r] == n
        rt, rix = orc.kd_build(coords[r, cols])
        if (tcol[r, :n] == cols).all() and tree[r, :n].tobytes() == coords[r, cols].tobytes():
            # left in column order (or rebuilt into a tree that is that order)
            assert nb[r] == 0 or rt.tobytes() == coords[r, cols].tobytes(), r
        else:
            assert nb[r] == 1, r
            rebuilt += 1
            _eq(tree[r, :n], rt, f"row {r} rebuilt tree")
            _eq(tcol[r, :n], cols[rix], f"row {r} rebuilt cols")
        for c in np.nonzero(qm[r] == 1)[0]:
            p, d = orc.kd_nn(rt, lid2[r, c])
            assert (pos[r, c] >= 0) == (p >= 0) and dist[r, c] == d, (r, c)
            if p >= 0:
                assert tree[r, pos[r, c]].tobytes() == rt[p].tobytes(), (r, c)
        assert (pos[r][qm[r] == 0] == -1).all()
    if integer_mm:
        assert rebuilt > 0, rebuilt


@pytest.mark.parametrize("seed,integer_mm", [(5, True), (9, True), (5, False)])
def test_lazy_rows_fused_corr_equals_separate(gpu, seed, integer_mm):
    """kd_query_rows_lazy_corr_dev (the fast mode's row sums in the tie
    pass's launch, r5) against kd_query_rows_lazy_dev + rows_corr_dev on the
    same compacted rows: positions, distances, rebuilt rows and the six sums
    per row bit-identical, with ties (integer-mm, most rows rebuilt) and
    without."""
    import torch
    from navslam.synth import l9_pair
    R, Cc = 128, 2048
    lid, lid2 = l9_pair(R, Cc, seed=seed, integer_mm=integer_mm)
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_lid, d_lid2 = t(lid), t(lid2)
    ori = t(lid2 + np.array([3.0, -1.0, 0.5]))
    out = {}
    for fused in (False, True):
        tree = torch.zeros((R, Cc, 3), dtype=torch.float64, device=dev)
        tcol = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
        tn = torch.zeros(R, dtype=torch.int32, device=dev)
        built = torch.zeros(R, dtype=torch.int32, device=dev)
        pos = torch.zeros((R, Cc), dtype=torch.int32, device=dev)
        dist = torch.zeros((R, Cc), dtype=torch.float64, device=dev)
        sums = torch.zeros((R, 6), dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        gpu.kd_compact_rows_dev(d_lid, d_lid, R, Cc, tree, tcol, tn, None, built)
        if fused:
            gpu.kd_query_rows_lazy_corr_dev(tree, tcol, tn, d_lid2, d_lid2, R, Cc, pos, dist,
                                            None, built, ori, sums)
        else:
            gpu.kd_query_rows_lazy_dev(tree, tcol, tn, d_lid2, d_lid2, R, Cc, pos, dist,
                                       None, built)
            gpu.rows_corr_dev(tree, tn, pos, dist, ori, R, Cc, None, sums)
        gpu.sync()
        out[fused] = [x.cpu().numpy() for x in (tree, tcol, built, pos, dist, sums)]
    for a, b, nm in zip(out[False], out[True], ("tree", "cols", "built", "pos", "dist", "sums")):
        _eq(b, a, nm)
    if integer_mm:
        assert out[True][2].sum() > 0  # some rows met a tie and were rebuilt


def test_lazy_rows_refused_fused_call_leaves_context_clean(gpu, orc):
    """a fused lazy call the library refuses (C = 2100: its hash
    table needs more LDS than a workgroup has) must not leave tie flags
    behind. Rows built by an earlier lazy query (built = 1) are then walked
    as they stand by the next valid query on the same context, not rebuilt
    from tree order: trees, positions and distances unchanged, and equal to
    the oracle's KD walk."""
    import torch
    from navslam.gpu import NavGpuError
    from navslam.synth import l9_pair
    R, Cc = 8, 2048
    lid, lid2 = l9_pair(R, Cc, seed=5, integer_mm=True)
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_lid, d_lid2 = t(lid), t(lid2)
    z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=dev)
    tree, tcol = z((R, Cc, 3), torch.float64), z((R, Cc), torch.int32)
    tn, built = z(R, torch.int32), z(R, torch.int32)
    pos, dist = z((R, Cc), torch.int32), z((R, Cc), torch.float64)
    torch.cuda.synchronize()
    gpu.kd_compact_rows_dev(d_lid, d_lid, R, Cc, tree, tcol, tn, None, built)
    gpu.kd_query_rows_lazy_dev(tree, tcol, tn, d_lid2, d_lid2, R, Cc, pos, dist, None, built)
    gpu.sync()
    assert built.sum().item() > 0  # integer-mm: some rows met a tie and hold their tree
    tree1, tcol1, pos1, dist1 = tree.clone(), tcol.clone(), pos.clone(), dist.clone()
    # the refused call: tie-heavy rows of 2100 columns, fused correspondences
    C2 = 2100
    a2, b2 = l9_pair(R, C2, seed=9, integer_mm=True)
    e_tree, e_col = z((R, C2, 3), torch.float64), z((R, C2), torch.int32)
    e_tn, e_built = z(R, torch.int32), z(R, torch.int32)
    gpu.kd_compact_rows_dev(t(a2), t(a2), R, C2, e_tree, e_col, e_tn, None, e_built)
    gpu.sync()
    with pytest.raises(NavGpuError):
        gpu.kd_query_rows_lazy_corr_dev(e_tree, e_col, e_tn, t(b2), t(b2), R, C2,
                                        z((R, C2), torch.int32), z((R, C2), torch.float64),
                                        None, e_built, t(b2), z((R, 6), torch.float64))
    gpu.sync()
    gpu.kd_query_rows_lazy_dev(tree, tcol, tn, d_lid2, d_lid2, R, Cc, pos, dist, None, built)
    gpu.sync()
    _eq(tree.cpu().numpy(), tree1.cpu().numpy(), "after the refused call: rows unchanged")
    _eq(tcol.cpu().numpy(), tcol1.cpu().numpy(), "after the refused call: columns unchanged")
    _eq(pos.cpu().numpy(), pos1.cpu().numpy(), "after the refused call: positions")
    _eq(dist.cpu().numpy(), dist1.cpu().numpy(), "after the refused call: distances")
    fm, qm = orc.extract_feature(lid), orc.extract_feature(lid2)
    tr, tnn, ps, ds = (x.cpu().numpy() for x in (tree, tn, pos, dist))
    for r in range(R):
        rt, _ = orc.kd_build(lid[r, np.nonzero(fm[r] == 1)[0]])
        for c in np.nonzero(qm[r] == 1)[0]:
            p, d = orc.kd_nn(rt, lid2[r, c])
            assert ds[r, c] == d, (r, c)
            if p >= 0:
                assert tr[r, ps[r, c]].tobytes() == rt[p].tobytes(), (r, c)


# ---------------------------------------------------------- global k-NN
@pytest.mark.parametrize("k", [1, 3, 8, 16])
def test_knn_vs_brute(kgpu, orc, k):
    rng = np.random.default_rng(k)
    for tgt, q in [(rng.uniform(0, 1000, (5000, 3)), rng.uniform(-50, 1050, (3000, 3))),
                   (np.round(rng.uniform(0, 20, (4000, 3))), np.round(rng.uniform(0, 20, (2000, 3)))),
                   (rng.uniform(0, 1, (7, 3)), rng.uniform(0, 1, (50, 3))),       # nt < k
                   (np.zeros((100, 3)), rng.uniform(-1, 1, (40, 3))),             # identical
                   (np.c_[rng.uniform(0, 100, 3000), np.zeros(3000), np.zeros(3000)],
                    rng.uniform(0, 100, (500, 3))),                              # degenerate axis
                   (np.zeros((0, 3)), rng.uniform(0, 1, (10, 3)))]:               # empty target
        ri, rd = orc.knn_brute(tgt, q, k)
        gi, gd = kgpu.knn(tgt, q, k)
        _eq(gi, ri, f"k={k} idx n={len(tgt)}")
        _eq(gd, rd, f"k={k} dist n={len(tgt)}")


def test_knn_error_flag_stays_clear(kgpu):
    """Every k-NN kernel clamps the list, cloud and record indices it loads
    through (so a logic error cannot fault the device) and flags the call
    when a clamp changed one (navgpu_knn_check -> NAVGPU_EINTERNAL). The
    small, degenerate and LDS-overflow inputs must leave it clear, through
    the device entry point (navgpu_knn_host checks it itself)."""
    import torch
    rng = np.random.default_rng(7)
    dev = torch.device("cuda", 0)
    cases = [(rng.uniform(0, 1000, (5000, 3)), rng.uniform(-50, 1050, (3000, 3))),
             (rng.uniform(0, 1, (7, 3)), rng.uniform(0, 1, (50, 3))),
             (np.zeros((100, 3)), rng.uniform(-1, 1, (40, 3))),
             (np.zeros((3000, 3)), np.zeros((300, 3))),          # one overfull cell
             (np.c_[rng.uniform(0, 100, 3000), np.zeros(3000), np.zeros(3000)],
              rng.uniform(0, 100, (500, 3))),
             (np.zeros((0, 3)), rng.uniform(0, 1, (10, 3))),
             (_clustered(rng, 20000, 6, 0.5, 1000.0), rng.uniform(0, 1000, (4000, 3)))]
    for t, q in cases:
        tt = torch.from_numpy(np.ascontiguousarray(t)).to(dev)
        qq = torch.from_numpy(np.ascontiguousarray(q)).to(dev)
        for k in (1, 8):
            idx = torch.empty((len(q), k), dtype=torch.int32, device=dev)
            dst = torch.empty((len(q), k), dtype=torch.float64, device=dev)
            kgpu.knn_dev(tt if len(t) else qq, len(t), qq, len(q), k, idx, dst)
            kgpu.knn_check()


def _clustered(rng, n, centers, sigma, box):
    c = rng.uniform(0, box, (centers, 3))
    pts = c[rng.integers(0, centers, n)] + rng.normal(0, sigma, (n, 3))
    return np.concatenate([pts, rng.uniform(0, box, (n // 10, 3))])


@pytest.mark.parametrize("k", [1, 8])
def test_knn_hard_cases(kgpu, orc, k):
    """Inputs that leave the fast path: dense clusters (LDS-overflow tiles,
    runs longer than a key's offset field), non-finite coordinates, queries
    far outside the target box, a large common offset."""
    rng = np.random.default_rng(100 + k)
    cases = []
    # dense clusters in a sparse box: grid sized by the mean density
    t = _clustered(rng, 20000, 6, 0.5, 1000.0)
    q = np.concatenate([_clustered(rng, 3000, 6, 0.5, 1000.0), rng.uniform(0, 1000, (500, 3))])
    cases.append(("clusters", t, q))
    # non-finite targets and queries: never a neighbour / no neighbours
    t = rng.uniform(0, 100, (3000, 3))
    t[rng.integers(0, 3000, 40), rng.integers(0, 3, 40)] = np.nan
    t[rng.integers(0, 3000, 40), rng.integers(0, 3, 40)] = np.inf
    t[rng.integers(0, 3000, 20), rng.integers(0, 3, 20)] = -np.inf
    q = rng.uniform(-10, 110, (800, 3))
    q[rng.integers(0, 800, 30), rng.integers(0, 3, 30)] = np.nan
    q[rng.integers(0, 800, 30), rng.integers(0, 3, 30)] = np.inf
    cases.append(("non-finite", t, q))
    # queries far outside the target box (every one needs the exact search)
    t = rng.uniform(0, 100, (4000, 3))
    q = rng.uniform(0, 100, (300, 3)) + np.array([1e5, 0, 0]) * rng.choice([-1, 1], (300, 1))
    cases.append(("far queries", t, q))
    # large common offset (f32 keys are relative to the grid origin)
    off = np.array([3.7e6, -1.2e6, 9.9e5])
    t = rng.uniform(0, 50, (4000, 3)) + off
    q = rng.uniform(-2, 52, (1500, 3)) + off
    cases.append(("offset", t, q))
    for name, tgt, qs in cases:
        ri, rd = orc.knn_brute(tgt, qs, k)
        gi, gd = kgpu.knn(tgt, qs, k)
        _eq(gi, ri, f"{name} k={k} idx")
        _eq(gd, rd, f"{name} k={k} dist")


@pytest.mark.parametrize("mode", KNN_MODES)
@pytest.mark.parametrize("sx", [1, 2, 3, 8])
def test_knn_cell_slicing_variants(orc, sx, mode, monkeypatch):
    """NAVGPU_KNN_SX (x cells per h; default 3) reshapes every tile, block
    and certificate reach: each setting gives the brute-force answer, on
    uniform, integer-mm and clustered data, k = 2, 8 and 13."""
    from navslam.gpu import NavGpu
    monkeypatch.setenv("NAVGPU_KNN_SX", str(sx))
    monkeypatch.setenv("NAVGPU_KNN_MODE", str(mode))
    g = NavGpu(0)
    try:
        rng = np.random.default_rng(40 + sx)
        cases = [(rng.uniform(0, 800, (6000, 3)), rng.uniform(-20, 820, (2500, 3))),
                 (np.round(rng.uniform(0, 30, (5000, 3))), np.round(rng.uniform(0, 30, (1500, 3)))),
                 (_clustered(rng, 8000, 4, 1.0, 500.0), rng.uniform(0, 500, (1200, 3)))]
        for ci, (t, q) in enumerate(cases):
            for k in (2, 8, 13):
                ri, rd = _memo(("sx", sx, ci, k), lambda: orc.knn_brute(t, q, k))
                gi, gd = g.knn(t, q, k)
                _eq(gi, ri, f"sx={sx} case {ci} k={k} idx")
                _eq(gd, rd, f"sx={sx} case {ci} k={k} dist")
    finally:
        g.close()


def test_knn_huge_coordinates(kgpu, orc):
    """Coordinates past the f32 offsets' certified range (|x| ~ 1e18 mm) and a
    cloud spanning 1e-3 .. 1e15 mm: the certificate fails and the slow path
    answers, exactly."""
    rng = np.random.default_rng(77)
    t = rng.uniform(-1, 1, (2000, 3)) * 1e18
    q = rng.uniform(-1, 1, (300, 3)) * 1e18
    ri, rd = orc.knn_brute(t, q, 8)
    gi, gd = kgpu.knn(t, q, 8)
    _eq(gi, ri, "1e18 idx")
    _eq(gd, rd, "1e18 dist")
    t = np.concatenate([rng.uniform(0, 1e-3, (1500, 3)), rng.uniform(0, 1e15, (1500, 3))])
    q = np.concatenate([rng.uniform(0, 1e-3, (200, 3)), rng.uniform(0, 1e15, (200, 3))])
    ri, rd = orc.knn_brute(t, q, 4)
    gi, gd = kgpu.knn(t, q, 4)
    _eq(gi, ri, "wide-range idx")
    _eq(gd, rd, "wide-range dist")


def test_knn_k1_agrees_with_reference_kd_distances(kgpu, golden):
    for pts, perm, q, nn, nnd in _golden_sets(golden("kdtree")):
        if len(pts) == 0:
            continue
        gi, gd = kgpu.knn(pts, q, 1)
        _eq(gd[:, 0], nnd, "1-NN distance vs reference KD")


def test_knn_k3_full_size_all_queries(kgpu, orc):
    """K3 at full size (1M x 1M, k=8): EVERY query against the oracle's exact
    grid k-NN (orc_knn_grid, pinned to the brute force by test_oracle.py),
    plus a seeded sample of 1024 against the brute force itself."""
    from navslam.synth import uniform_pair
    src, tgt = uniform_pair(512, 2048)
    gi, gd = kgpu.knn(tgt, src, 8)
    ri, rd = _memo("k3", lambda: orc.knn_grid(tgt, src, 8))
    _eq(gi, ri, "all 1M queries: idx")
    _eq(gd, rd, "all 1M queries: dist")
    s = np.random.default_rng(9).choice(len(gi), 1024, replace=False)
    bi, bd = _memo("k3b", lambda: orc.knn_brute(tgt, src.reshape(-1, 3)[s], 8))
    _eq(gi[s], bi, "sampled idx vs brute force")
    _eq(gd[s], bd, "sampled dist vs brute force")


@pytest.mark.parametrize("integer_mm", [False, True])
def test_knn_global_on_l9_scan(kgpu, orc, integer_mm):
    """Global mode on a lidar-shaped pair instead of the uniform K3 cloud:
    points on surfaces (most grid cells empty, the rest dense), 2 % dropouts
    that all sit at (0, 0, 0) (utils/pointcloud.c:24-27: one cell holding
    thousands of identical points, so LDS-overflow tiles, overfull runs and
    the slow path with massive distance ties), and integer-mm coordinates.
    Every query against the oracle's exact grid k-NN."""
    from navslam.synth import l9_pair
    src, tgt = l9_pair(128, 2048, seed=21, integer_mm=integer_mm)
    for k in (1, 8):
        gi, gd = kgpu.knn(tgt, src, k)
        ri, rd = _memo(("l9", integer_mm, k), lambda: orc.knn_grid(tgt, src, k))
        _eq(gi, ri, f"l9 integer_mm={integer_mm} k={k}: idx")
        _eq(gd, rd, f"l9 integer_mm={integer_mm} k={k}: dist")


def _degenerate_clouds(name, rng):
    n = 200_000
    if name == "line":  # one grid axis at its 2048-cell cap, the others 1 cell
        t = np.c_[rng.uniform(0, 1e4, n), rng.normal(0, 1e-3, n), np.zeros(n)]
        q = np.c_[rng.uniform(-10, 1e4 + 10, 50_000), rng.normal(0, 1, 50_000),
                  rng.normal(0, 1, 50_000)]
    elif name == "plane":  # a flat target, queries above and below it
        t = np.c_[rng.uniform(0, 1e3, n), rng.uniform(0, 1e3, n), np.zeros(n)]
        q = np.c_[rng.uniform(0, 1e3, 50_000), rng.uniform(0, 1e3, 50_000),
                  rng.normal(0, 5, 50_000)]
    else:  # two dense clusters 1e6 mm apart: almost every cell empty
        t = np.concatenate([rng.normal(0, 10, (n // 2, 3)), rng.normal(1e6, 10, (n // 2, 3))])
        q = np.concatenate([rng.normal(0, 12, (25_000, 3)), rng.normal(1e6, 12, (25_000, 3)),
                            rng.uniform(0, 1e6, (1_000, 3))])
    return t, q


@pytest.mark.parametrize("name", ["line", "plane", "far_clusters"])
def test_knn_global_degenerate_distributions(kgpu, orc, name):
    """Distributions the uniform grid handles worst (overflow tiles, overfull
    runs, a slow path for most queries, rings across empty space): every
    query against the oracle's exact grid k-NN, k = 8."""
    t, q = _degenerate_clouds(name, np.random.default_rng(5))
    gi, gd = kgpu.knn(t, q, 8)
    ri, rd = _memo(("degenerate", name), lambda: orc.knn_grid(t, q, 8))
    _eq(gi, ri, f"{name}: idx")
    _eq(gd, rd, f"{name}: dist")


def _digest_inputs_match(dg, prefix, src, tgt):
    from golden.make_golden import sha
    if sha(src) != str(dg[prefix + "_src"]) or sha(tgt) != str(dg[prefix + "_tgt"]):
        pytest.fail(f"{prefix}: the synthetic input differs from the one the reference "
                    "digests were made from (numpy on this host generates other values)")


def test_knn_k1_1m_matches_reference_kd_digest(kgpu, golden):
    """the reference's own buildKDTree + nearestNeighborSearch over
    the 1M K3 pair (oracle/_ref, digests made by tests/golden/make_golden.py):
    the GPU's 1-NN points and distances hash to the same SHA-256."""
    from golden.make_golden import nn_digest_arrays, sha
    from navslam.synth import uniform_pair
    dg = golden("digests")
    src, tgt = uniform_pair(512, 2048)
    _digest_inputs_match(dg, "k3", src, tgt)
    gi, gd = kgpu.knn(tgt, src, 1)
    pts, d = nn_digest_arrays(tgt.reshape(-1, 3), gi[:, 0], gd[:, 0])
    _eq(pts[:64], dg["k3_head_nn"], "first 64 nearest points")
    _eq(d[:64], dg["k3_head_nnd"], "first 64 distances")
    assert sha(pts) == str(dg["k3_nn"]), "1M nearest points differ from the reference KD"
    assert sha(d) == str(dg["k3_nnd"]), "1M distances differ from the reference KD"


@pytest.mark.parametrize("tag,integer", [("f", False), ("i", True)])
def test_rows_match_k2_matches_reference_digest(gpu, golden, tag, integer):
    """the K2 128x2048 pair in per-row mode against the reference's
    per-row buildKDTree + nearestNeighborSearch (digests of the nearest
    points and distances of every source feature, row-major)."""
    from golden.make_golden import nn_digest_arrays, sha
    from navslam.synth import l9_pair
    dg = golden("digests")
    src, tgt = l9_pair(128, 2048, seed=5, integer_mm=integer)
    _digest_inputs_match(dg, "k2" + tag, src, tgt)
    sm, tm, idx, dist = gpu.rows_match(src, tgt)
    assert sha(sm) == str(dg[f"k2{tag}_smask"]) and sha(tm) == str(dg[f"k2{tag}_tmask"])
    q = sm.reshape(-1) == 1
    assert int(q.sum()) == int(dg[f"k2{tag}_nq"])
    pts, d = nn_digest_arrays(tgt.reshape(-1, 3), idx.reshape(-1)[q], dist.reshape(-1)[q])
    assert sha(pts) == str(dg[f"k2{tag}_nn"]), "nearest points differ from the reference"
    assert sha(d) == str(dg[f"k2{tag}_nnd"]), "distances differ from the reference"


@pytest.mark.parametrize("C", [1, 2, 3, 4, 5, 6, 59, 60, 61, 63, 64, 65, 119, 120, 121, 241, 1000])
def test_curvature_segment_edges(gpu, orc, C):
    """k_curvature covers a row with waves of 60 output columns and a
    2-column halo: row widths around the segment and block edges (and rows
    too short for any curvature) against the oracle."""
    rng = np.random.default_rng(C)
    pts = rng.uniform(-2000, 2000, (5, C, 3))
    pts[1] = np.round(pts[1])
    m_ref, c_ref = orc.extract_feature(pts, want_curv=True)
    m, cv = gpu.curvature(pts, want_curv=True)
    _eq(m, m_ref, f"C={C} mask")
    _eq(cv, c_ref, f"C={C} curvature")


def test_curvature_k3_shape_bit_exact(gpu, orc):
    """R1 at the K3 shape: both 512x2048 clouds, mask and f64 value."""
    from navslam.synth import uniform_pair
    for pts in uniform_pair(512, 2048):
        m_ref, c_ref = orc.extract_feature(pts, want_curv=True)
        m, cv = gpu.curvature(pts, want_curv=True)
        _eq(m, m_ref, "512x2048 mask")
        _eq(cv, c_ref, "512x2048 curvature")


# ------------------------------------------------------- slam.h drop-in
def _run_shim_stream(shim, depth, imu, use_gpu_project=True):
    from pyoracle import Oracle, OracleEkf
    orc = Oracle()
    from shimlib import Pos, preorder
    to_pos = lambda v: np.array([v[0] * 1000, v[1] * 1000, v[2] * 1000, v[3], v[4], v[5]])
    R, Cc = shim.R, shim.C
    attr = shim.SLAMAttr()

    def cloud(d):
        if use_gpu_project:
            pts = np.zeros((R, Cc, 3))
            dd = np.ascontiguousarray(d, np.int32)
            shim.L.convertToPointCloud(dd.ctypes.data, pts.ctypes.data)
            return pts
        return orc.convert(d)

    pos = to_pos(imu[0])
    ekf = OracleEkf(orc, pos)
    shim.L.init_slam(C.byref(attr), Pos.of(pos), C.byref(shim.cloud(cloud(depth[0]))))
    out = {"meas": [], "fused": [], "err": [], "trees": []}
    out["trees"].append([preorder(attr.kdtree_lastframe[r]) for r in range(R)])
    last = pos
    for i in range(1, len(depth)):
        ekf.predict(to_pos(imu[i - 1]), to_pos(imu[i]))
        pred = ekf.pos
        pc = shim.cloud(cloud(depth[i]))
        meas = shim.L.slam_localization(C.byref(attr), C.byref(pc), Pos.of(pred), Pos.of(last))
        ekf.update_R(attr.error)
        ekf.modify(np.array(meas.tolist()))
        fused = ekf.pos
        shim.L.slam_mapping(C.byref(attr), Pos.of(fused), C.byref(pc))
        out["meas"].append(meas.tolist())
        out["fused"].append(list(fused))
        out["err"].append(attr.error)
        out["trees"].append([preorder(attr.kdtree_lastframe[r]) for r in range(R)])
        last = fused
    out["frame_count"] = attr.frameCount
    n = attr.frameCount - 1
    out["last_global"] = np.frombuffer(bytes(attr.globalPointCloud[n % 100].pos),
                                       np.float64).reshape(R, Cc, 3)
    return out


def test_shim_l5_stream_matches_reference_golden(golden, monkeypatch):
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    from shimlib import Shim
    g = golden("slam8x8")
    out = _run_shim_stream(Shim(8, 8), g["depth"], g["imu"])
    _eq(np.array(out["meas"]), g["pos_meas"], "pos_measure trace")
    _eq(np.array(out["fused"]), g["pos_fused"], "fused pose trace")
    _eq(np.array(out["err"]), g["error"], "registration error")
    assert out["frame_count"] == int(g["frame_count"])
    _eq(out["last_global"], g["last_global"], "globalPointCloud")
    off = 0
    for f, fr in enumerate(g["tree_n"]):
        for r, n in enumerate(fr):
            _eq(np.array(out["trees"][f][r]).reshape(-1, 3),
                g["tree_pts"][off:off + n].reshape(-1, 3), f"tree frame {f} row {r}")
            off += n


def test_shim_l5_stream_lazy_rows_match_reference_golden(golden, monkeypatch):
    """The same golden trace with NAVSLAM_HOST_TREES=0 (no KDNode trees
    handed out; the device rows hold compacted features and a row gets its
    tree only when a query meets a distance tie): poses, errors and the map
    unchanged, kdtree_lastframe left NULL."""
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    monkeypatch.setenv("NAVSLAM_HOST_TREES", "0")
    from shimlib import Shim
    g = golden("slam8x8")
    out = _run_shim_stream(Shim(8, 8), g["depth"], g["imu"])
    _eq(np.array(out["meas"]), g["pos_meas"], "pos_measure trace")
    _eq(np.array(out["fused"]), g["pos_fused"], "fused pose trace")
    _eq(np.array(out["err"]), g["error"], "registration error")
    assert out["frame_count"] == int(g["frame_count"])
    _eq(out["last_global"], g["last_global"], "globalPointCloud")
    assert all(len(t) == 0 for fr in out["trees"] for t in fr)


@pytest.mark.parametrize("trees", ["1", "0"])
@pytest.mark.parametrize("R,Cc,frames", [(54, 42, 12), (128, 2048, 4)])
def test_shim_stream_vs_oracle(monkeypatch, R, Cc, frames, trees):
    """Larger grids (L9 54x42, K2 128x2048): shim vs the oracle frame loop,
    with the host KDNode trees built every frame (NAVSLAM_HOST_TREES=1) and
    with the lazy device rows (=0: compacted rows, a tree only for a row whose
    screen met a distance tie)."""
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    monkeypatch.setenv("NAVSLAM_HOST_TREES", trees)
    from pyoracle import Oracle, OracleEkf, OracleSlam
    from shimlib import Shim
    orc = Oracle()
    rng = np.random.default_rng(R)
    from navslam.synth import l5_stream
    depth8, imu = l5_stream(rng, frames)
    # widen the 8x8 scene to R x C by nearest resampling + noise
    ri = (np.arange(R) * 8 // R)
    ci = (np.arange(Cc) * 8 // Cc)
    depth = depth8[:, ri][:, :, ci] + rng.integers(-3, 4, (frames, R, Cc))
    got = _run_shim_stream(Shim(R, Cc), depth, imu, use_gpu_project=True)
    to_pos = lambda v: np.array([v[0] * 1000, v[1] * 1000, v[2] * 1000, v[3], v[4], v[5]])
    pos = to_pos(imu[0])
    ekf = OracleEkf(orc, pos)
    s = OracleSlam(orc, R, Cc)
    s.init(pos, orc.convert(depth[0]))
    last = pos
    for i in range(1, frames):
        ekf.predict(to_pos(imu[i - 1]), to_pos(imu[i]))
        pred = ekf.pos
        cl = orc.convert(depth[i])
        meas, _, _ = s.localization(cl, pred, last)
        _eq(np.array(got["meas"][i - 1]), meas, f"frame {i} measurement")
        assert got["err"][i - 1] == s.error
        ekf.update_R(s.error)
        ekf.modify(meas)
        fused = ekf.pos
        s.mapping(fused, cl)
        last = fused
    _eq(got["last_global"], s.last_global(), "last global frame")


@pytest.mark.parametrize("trees", ["1", "0"])
@pytest.mark.parametrize("R,Cc,F,steps", [(54, 42, 4, 9), (128, 2048, 3, 4)])
def test_shim_l9_stream_vs_oracle(monkeypatch, R, Cc, F, steps, trees):
    """K5 shape: the L9 loop of src/main.c:423-431 (localization with
    pred = last, then mapping at the measured pose) over a ray-cast stream
    replayed back and forth, through the drop-in ABI; every pose, error and
    the frame stats bit-exact against the oracle's slam.c restatement, with
    host trees on and off (lazy rows)."""
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    monkeypatch.setenv("NAVSLAM_HOST_TREES", trees)
    from pyoracle import Oracle, OracleSlam
    from shimlib import Pos, Shim
    from navslam.synth import l9_stream, l9_stream_index
    frames = l9_stream(R, Cc, F, seed=17)
    sh = Shim(R, Cc)
    attr = sh.SLAMAttr()
    pcs = [sh.cloud(f) for f in frames]
    zero = np.zeros(6)
    sh.L.init_slam(C.byref(attr), Pos.of(zero), C.byref(pcs[0]))
    orc = Oracle()
    s = OracleSlam(orc, R, Cc)
    s.init(zero, frames[0])
    last_g, last_o = Pos.of(zero), zero
    for i in range(1, steps + 1):
        f = l9_stream_index(i, F)
        meas = sh.L.slam_localization(C.byref(attr), C.byref(pcs[f]), last_g, last_g)
        sh.L.slam_mapping(C.byref(attr), meas, C.byref(pcs[f]))
        om, iters, ncp = s.localization(frames[f], last_o, last_o)
        s.mapping(om, frames[f])
        _eq(np.array(meas.tolist()), om, f"frame {i} pose")
        assert attr.error == s.error, f"frame {i} error"
        q, cp, it = sh.last_frame_stats()
        assert (cp, it) == (ncp, iters), f"frame {i} stats {(cp, it)} vs {(ncp, iters)}"
        assert q >= cp
        last_g, last_o = meas, om
    assert attr.frameCount == s.frame_count


@pytest.mark.parametrize("d2h,trees", [("0", "0"), ("1", "0"), ("0", "1"), ("1", "1")])
def test_shim_copy_paths_vs_oracle(monkeypatch, d2h, trees):
    """Both ways the map slot comes back (NAVSLAM_D2H: 0 on the main stream
    after the row trees / compaction, 1 on the side stream during them), with
    host trees and lazy rows, on the K5 loop at 128 x 2048 (6.3 MB per
    slot): every map slot and pose bit-exact against the oracle."""
    monkeypatch.setenv("NAVSLAM_D2H", d2h)
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    monkeypatch.setenv("NAVSLAM_HOST_TREES", trees)
    from pyoracle import Oracle, OracleSlam
    from shimlib import Pos, Shim
    from navslam.synth import l9_stream, l9_stream_index
    R, Cc, F = 128, 2048, 3
    frames = l9_stream(R, Cc, F, seed=23)
    sh = Shim(R, Cc)
    attr = sh.SLAMAttr()
    pcs = [sh.cloud(f) for f in frames]
    zero = np.zeros(6)
    sh.L.init_slam(C.byref(attr), Pos.of(zero), C.byref(pcs[0]))
    s = OracleSlam(Oracle(), R, Cc)
    s.init(zero, frames[0])
    slot = lambda n: np.frombuffer(bytes(attr.globalPointCloud[n % 100].pos),
                                   np.float64).reshape(R, Cc, 3)
    _eq(slot(0), s.last_global(), "map slot 0")
    last_g, last_o = Pos.of(zero), zero
    for i in range(1, 5):
        f = l9_stream_index(i, F)
        meas = sh.L.slam_localization(C.byref(attr), C.byref(pcs[f]), last_g, last_g)
        sh.L.slam_mapping(C.byref(attr), meas, C.byref(pcs[f]))
        om, _, _ = s.localization(frames[f], last_o, last_o)
        s.mapping(om, frames[f])
        _eq(np.array(meas.tolist()), om, f"frame {i} pose")
        _eq(slot(attr.frameCount - 1), s.last_global(), f"map slot {i}")
        last_g, last_o = meas, om


@pytest.mark.parametrize("trees,adam", [("1", "exact"), ("0", "exact"), ("0", "fast")])
def test_shim_localise_twice_between_mappings(monkeypatch, trees, adam):
    """Two localisations against the same map (no slam_mapping between them,
    a caller the reference allows): with lazy rows (NAVSLAM_HOST_TREES=0) the
    first call turns tied rows into the reference tree in place, and the
    second must walk that tree, not rebuild one from the permuted order
    (ADVICE r4). Integer-mm frames make ties common. Every pose and error
    against the oracle's slam.c, for host trees on and off; in fast mode
    (the fused lazy query + row sums) the correspondence counts
    exactly and the poses within the fast mode's 1e-6."""
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    monkeypatch.setenv("NAVSLAM_HOST_TREES", trees)
    if adam == "fast":
        monkeypatch.setenv("NAVSLAM_ADAM", "fast")
    else:
        monkeypatch.delenv("NAVSLAM_ADAM", raising=False)
    from pyoracle import Oracle, OracleSlam
    from shimlib import Pos, Shim
    from navslam.synth import l9_stream
    R, Cc, F = 128, 2048, 4
    frames = l9_stream(R, Cc, F, seed=29, integer_mm=True)
    sh = Shim(R, Cc)
    attr = sh.SLAMAttr()
    pcs = [sh.cloud(f) for f in frames]
    zero = np.zeros(6)
    sh.L.init_slam(C.byref(attr), Pos.of(zero), C.byref(pcs[0]))
    orc = Oracle()
    s = OracleSlam(orc, R, Cc)
    s.init(zero, frames[0])
    last_g, last_o = Pos.of(zero), zero
    for f in range(1, F):
        for rep in range(2):  # the same map twice; the second starts at the first's answer
            meas = sh.L.slam_localization(C.byref(attr), C.byref(pcs[f]), last_g, last_g)
            om, _, ncp = s.localization(frames[f], last_o, last_o)
            if adam == "fast":
                np.testing.assert_allclose(np.array(meas.tolist()), om, rtol=0, atol=1e-6,
                                           err_msg=f"frame {f} localisation {rep} pose")
                assert sh.last_frame_stats()[1] == ncp, f"frame {f} localisation {rep}"
                assert abs(attr.error - s.error) <= 1e-9 * max(1.0, s.error)
                # (the chain continues from the oracle's pose, so both sides
                # localise the same frame from the same start)
                meas = Pos.of(om)
            else:
                _eq(np.array(meas.tolist()), om, f"frame {f} localisation {rep} pose")
                assert attr.error == s.error, f"frame {f} localisation {rep} error"
            last_g, last_o = meas, om
        sh.L.slam_mapping(C.byref(attr), meas, C.byref(pcs[f]))
        s.mapping(om, frames[f])


def _dedup_reference(orc, tree, pos, dist, ori):
    """src/slam.c:236-284 through the oracle's list builder (orc_rows_dedup,
    the code orc_slam_localization runs, pinned by the slam8x8 golden):
    the keep mask and per-row (sum d, centred sum |d - mean|^2, count,
    queries) over the listed pairs, d = ori - near."""
    R, Cc = pos.shape
    o, nr, _, g = orc.rows_dedup(tree, pos.astype(np.int64), dist, ori)
    keep = np.zeros(R * Cc, np.int32)
    keep[g] = 1
    sums = np.zeros((R, 6))
    rows = g // Cc
    d = o - nr
    for r in range(R):
        dr = d[rows == r]
        sums[r, :3] = dr.sum(axis=0)
        sums[r, 4] = len(dr)
        if len(dr):
            sums[r, 3] = ((dr - dr.mean(axis=0)) ** 2).sum()
        sums[r, 5] = (pos[r] >= 0).sum()
    return keep.reshape(R, Cc), sums


@pytest.mark.parametrize("integer_mm", [False, True])
def test_rows_corr_matches_reference_dedup(gpu, orc, integer_mm):
    """R7 on the GPU (navgpu_rows_corr_dev) against the reference list rule,
    on real per-row trees/queries; integer-mm coordinates make duplicate
    nearest points and distance ties common."""
    import torch
    from navslam.synth import l9_pair
    src, tgt = l9_pair(24, 640, seed=21, integer_mm=integer_mm)
    R, Cc = src.shape[:2]
    dev = torch.device("cuda", 0)
    ss, ts = torch.from_numpy(src).to(dev), torch.from_numpy(tgt).to(dev)
    tree = torch.empty_like(ts)
    tcol = torch.empty((R, Cc), dtype=torch.int32, device=dev)
    tn = torch.empty(R, dtype=torch.int32, device=dev)
    pos = torch.empty((R, Cc), dtype=torch.int32, device=dev)
    dist = torch.empty((R, Cc), dtype=torch.float64, device=dev)
    keep = torch.empty((R, Cc), dtype=torch.int32, device=dev)
    sums = torch.empty((R, 6), dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    gpu.kd_build_rows_dev(ts, ts, R, Cc, tree, tcol, tn)
    gpu.kd_query_rows_dev(tree, tn, ss, ss, R, Cc, pos, dist)
    gpu.rows_corr_dev(tree, tn, pos, dist, ss, R, Cc, keep, sums)
    gpu.sync()
    ek, es = _dedup_reference(orc, tree.cpu().numpy(), pos.cpu().numpy(),
                              dist.cpu().numpy(), src)
    _eq(keep.cpu().numpy(), ek, "kept correspondences")
    np.testing.assert_allclose(sums.cpu().numpy(), es, rtol=1e-12, atol=1e-9)
    assert ek.sum() > 0 and (ek.sum() < (pos.cpu().numpy() >= 0).sum() or not integer_mm)


@pytest.mark.parametrize("n", [400_000_000, 1 << 30])
def test_kd_build_beyond_limit_returns_erange(gpu, n):
    """navgpu_kd_build_dev (include/navgpu.h): above about 383M points a
    level holds more than 65535 windows (grid.y of the selection kernels),
    and n >= 2^30 overflows the int positions: both return NAVGPU_ERANGE
    (-4) before any workspace is sized for n or any point is read (ADVICE
    r2)."""
    import torch
    from navslam.gpu import NavGpuError
    pts = torch.zeros((4, 3), dtype=torch.float64, device="cuda")
    with pytest.raises(NavGpuError, match=r"\(-4\)"):
        gpu.kd_build_dev(pts, n)
    gpu.sync()


def test_rows_corr_rows_beyond_lds_return_erange(gpu):
    """The dedup kernels hold a row's hash (>= 2C slots) in LDS: rows wider
    than 2048 columns exceed the device's LDS and must return NAVGPU_ERANGE
    (-4) before any launch, not fail inside HIP."""
    import torch
    from navslam.gpu import NavGpuError
    R, Cc = 2, 2112
    dev = torch.device("cuda", 0)
    pts = torch.zeros((R, Cc, 3), dtype=torch.float64, device=dev)
    tn = torch.zeros(R, dtype=torch.int32, device=dev)
    pos = torch.full((R, Cc), -1, dtype=torch.int32, device=dev)
    dist = torch.full((R, Cc), float("inf"), dtype=torch.float64, device=dev)
    keep = torch.empty((R, Cc), dtype=torch.int32, device=dev)
    sums = torch.empty((R, 6), dtype=torch.float64, device=dev)
    with pytest.raises(NavGpuError, match=r"\(-4\)"):
        gpu.rows_corr_dev(pts, tn, pos, dist, pts, R, Cc, keep, sums)
    lst = torch.empty((R * Cc, 7), dtype=torch.float64, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    with pytest.raises(NavGpuError, match=r"\(-4\)"):
        gpu.rows_corr_list_dev(pts, tn, pos, dist, pts, R, Cc, lst, count)
    gpu.sync()


@pytest.mark.parametrize("R,Cc", [(24, 640), (2100, 42)])
def test_kd_rows_nodes_image_links_the_implicit_trees(gpu, R, Cc):
    """navgpu_kd_rows_nodes_dev: the KDNode image (utils/kdtree.h:7-11) of the
    row trees, with host addresses, links exactly the implicit layout of
    buildKDTree (node of [lo,hi) at lo+(hi-lo)/2, utils/kdtree.c:65-82); rows
    with no features give no nodes; 2100 rows take the offset scan past one
    row per thread."""
    import torch
    from navslam.synth import l9_pair
    _, tgt = l9_pair(R, Cc, seed=31)
    tgt[1] = 0.0  # a flat row: no features, an empty tree
    dev = torch.device("cuda", 0)
    ts = torch.from_numpy(tgt).to(dev)
    tree = torch.empty_like(ts)
    tcol = torch.empty((R, Cc), dtype=torch.int32, device=dev)
    tn = torch.empty(R, dtype=torch.int32, device=dev)
    off = torch.full((R + 1,), -1, dtype=torch.int32, device=dev)
    nodes = torch.empty((R * Cc, 5), dtype=torch.float64, device=dev)
    host = np.zeros((R * Cc, 5), np.float64)
    base = host.ctypes.data
    torch.cuda.synchronize()
    gpu.kd_build_rows_dev(ts, ts, R, Cc, tree, tcol, tn)
    gpu.kd_rows_nodes_dev(tree, tn, R, Cc, base, nodes, off)
    gpu.sync()
    tn, off, tree = tn.cpu().numpy(), off.cpu().numpy(), tree.cpu().numpy()
    assert tn[1] == 0 and (tn > 0).sum() > R // 2
    _eq(off, np.concatenate([[0], np.cumsum(tn)]).astype(np.int32), "row offsets")
    img = nodes.cpu().numpy()[: off[R]]
    pts, links = img[:, :3], img[:, 3:].copy().view(np.uint64)
    for r in range(R):
        o, n = int(off[r]), int(tn[r])
        _eq(pts[o:o + n], tree[r, :n], f"row {r} points")
        want = np.zeros((n, 2), np.uint64)
        stack = [(0, n)]
        while stack:
            lo, hi = stack.pop()
            mid = lo + (hi - lo) // 2
            for k, (a, b) in enumerate(((lo, mid), (mid + 1, hi))):
                if a < b:
                    want[mid, k] = base + 40 * (o + a + (b - a) // 2)
                    stack.append((a, b))
        _eq(links[o:o + n], want, f"row {r} links")


@pytest.mark.parametrize("integer_mm", [False, True])
def test_rows_corr_list_matches_reference_list(gpu, orc, integer_mm):
    """The exact mode's correspondence list built on the GPU
    (navgpu_rows_corr_list_dev) == the reference list (src/slam.c:235-284
    through orc_rows_dedup, pinned by the slam8x8 golden): same entries in
    the same order, bit for bit (oriPoint, nearestPoint, distance)."""
    import torch
    from navslam.synth import l9_pair
    src, tgt = l9_pair(24, 640, seed=23, integer_mm=integer_mm)
    src[3, 100:110] = np.nan  # NaN queries: no nearest point, no entry
    tgt[5, 50:60, 1] = np.nan  # NaN tree points: entries of their own
    R, Cc = src.shape[:2]
    dev = torch.device("cuda", 0)
    ss, ts = torch.from_numpy(src).to(dev), torch.from_numpy(tgt).to(dev)
    tree = torch.empty_like(ts)
    tcol = torch.empty((R, Cc), dtype=torch.int32, device=dev)
    tn = torch.empty(R, dtype=torch.int32, device=dev)
    pos = torch.empty((R, Cc), dtype=torch.int32, device=dev)
    dist = torch.empty((R, Cc), dtype=torch.float64, device=dev)
    lst = torch.full((R * Cc, 7), -7.0, dtype=torch.float64, device=dev)
    cnt = torch.zeros(2, dtype=torch.int32, device=dev)
    ori = ss + 0.25  # transformed frame (the oriPoint source)
    torch.cuda.synchronize()
    gpu.kd_build_rows_dev(ts, ts, R, Cc, tree, tcol, tn)
    gpu.kd_query_rows_dev(tree, tn, ss, ss, R, Cc, pos, dist)
    gpu.rows_corr_list_dev(tree, tn, pos, dist, ori, R, Cc, lst, cnt)
    gpu.sync()
    o, nr, d, _ = orc.rows_dedup(tree.cpu().numpy(), pos.cpu().numpy().astype(np.int64),
                                 dist.cpu().numpy(), ori.cpu().numpy())
    n, nq = (int(v) for v in cnt.cpu().numpy())
    assert n == len(d) and n > 0
    assert nq == int((pos.cpu().numpy() >= 0).sum())
    got = lst.cpu().numpy()[:n]
    _eq(got[:, 0:3], o, "oriPoint")
    _eq(got[:, 3:6], nr, "nearestPoint")
    _eq(got[:, 6], d, "distance")


@pytest.mark.parametrize("trees,lazy_corr", [("1", "1"), ("0", "1"), ("0", "0")])
@pytest.mark.parametrize("R,Cc,F,steps", [(54, 42, 4, 9), (128, 2048, 3, 4)])
def test_shim_l9_stream_fast_adam(monkeypatch, R, Cc, F, steps, trees, lazy_corr):
    """NAVSLAM_ADAM=fast (GPU dedup + closed-form Adam sums) on the K5 loop:
    the same correspondence counts as the oracle's slam.c restatement every
    frame, poses within 1e-6 mm / deg (tolerance of the order-free sums,
    which round differently from the reference's sequential ones). Lazy rows
    with the row sums fused into the tie pass (NAVSLAM_LAZY_CORR=1, default)
    and as a separate k_rows_corr launch into the pinned sums (=0)."""
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    monkeypatch.setenv("NAVSLAM_ADAM", "fast")
    monkeypatch.setenv("NAVSLAM_HOST_TREES", trees)
    monkeypatch.setenv("NAVSLAM_LAZY_CORR", lazy_corr)
    from pyoracle import Oracle, OracleSlam
    from shimlib import Pos, Shim
    from navslam.synth import l9_stream, l9_stream_index
    frames = l9_stream(R, Cc, F, seed=17)
    sh = Shim(R, Cc)
    attr = sh.SLAMAttr()
    pcs = [sh.cloud(f) for f in frames]
    zero = np.zeros(6)
    sh.L.init_slam(C.byref(attr), Pos.of(zero), C.byref(pcs[0]))
    s = OracleSlam(Oracle(), R, Cc)
    s.init(zero, frames[0])
    last_g, last_o = Pos.of(zero), zero
    for i in range(1, steps + 1):
        f = l9_stream_index(i, F)
        meas = sh.L.slam_localization(C.byref(attr), C.byref(pcs[f]), last_g, last_g)
        sh.L.slam_mapping(C.byref(attr), meas, C.byref(pcs[f]))
        om, iters, ncp = s.localization(frames[f], last_o, last_o)
        s.mapping(om, frames[f])
        np.testing.assert_allclose(np.array(meas.tolist()), om, rtol=0, atol=1e-6,
                                   err_msg=f"frame {i} pose")
        q, cp, it = sh.last_frame_stats()
        assert cp == ncp, f"frame {i}: {cp} correspondences vs {ncp}"
        assert abs(attr.error - s.error) <= 1e-9 * max(1.0, s.error)
        last_g, last_o = meas, om


@pytest.mark.parametrize("trees", ["1", "0"])
def test_shim_l9_long_stream_crosses_map_ring(monkeypatch, trees):
    """K5 past the reference's 100-frame map (headers/slam.h:12; src/slam.c:395
    writes globalPointCloud[frameCount] unbounded, the shim keeps a ring):
    the L9 loop at 54x42 for 120 frames, every pose, error and frame stat
    bit-exact against the oracle's slam.c restatement, frameCount past 100,
    and the ring slot of the last frame equal to the oracle's last map."""
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    monkeypatch.delenv("NAVSLAM_ADAM", raising=False)
    monkeypatch.setenv("NAVSLAM_HOST_TREES", trees)
    from pyoracle import Oracle, OracleSlam
    from shimlib import Pos, Shim
    from navslam.synth import l9_stream, l9_stream_index
    R, Cc, F, steps = 54, 42, 6, 120
    frames = l9_stream(R, Cc, F, seed=23)
    sh = Shim(R, Cc)
    attr = sh.SLAMAttr()
    pcs = [sh.cloud(f) for f in frames]
    zero = np.zeros(6)
    sh.L.init_slam(C.byref(attr), Pos.of(zero), C.byref(pcs[0]))
    s = OracleSlam(Oracle(), R, Cc)
    s.init(zero, frames[0])
    last_g, last_o = Pos.of(zero), zero
    for i in range(1, steps + 1):
        f = l9_stream_index(i, F)
        meas = sh.L.slam_localization(C.byref(attr), C.byref(pcs[f]), last_g, last_g)
        sh.L.slam_mapping(C.byref(attr), meas, C.byref(pcs[f]))
        om, iters, ncp = s.localization(frames[f], last_o, last_o)
        s.mapping(om, frames[f])
        _eq(np.array(meas.tolist()), om, f"frame {i} pose")
        assert attr.error == s.error, f"frame {i} error"
        q, cp, it = sh.last_frame_stats()
        assert (cp, it) == (ncp, iters), f"frame {i} stats"
        last_g, last_o = meas, om
    assert attr.frameCount == s.frame_count == steps + 1 > 100
    slot = (attr.frameCount - 1) % 100
    got = np.frombuffer(bytes(attr.globalPointCloud[slot].pos), np.float64).reshape(R, Cc, 3)
    _eq(got, s.last_global(), "ring slot of the last frame")


@pytest.mark.parametrize("offset", [(0.0, 0.0, 0.0), (1500.0, -700.0, 300.0),
                                    (2.5e5, 4.0e5, -1.0e5)])
def test_shim_fast_adam_error_finite_under_offset(monkeypatch, offset):
    """NAVSLAM_ADAM=fast with the map built at a shifted pose, so the residuals
    d = ori - near are large against their spread (the case where an
    uncentred closed form sum |d|^2 - 2 t.S1 + n |t|^2 cancels): the error
    stays finite and non-negative and matches the oracle's sequential sums.
    Offset 0 and the same frame: exact correspondences, error 0."""
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    monkeypatch.setenv("NAVSLAM_ADAM", "fast")
    from pyoracle import Oracle, OracleSlam
    from shimlib import Pos, Shim
    from navslam.synth import l9_stream
    R, Cc = 54, 42
    frames = l9_stream(R, Cc, 3, seed=29)
    sh = Shim(R, Cc)
    s = OracleSlam(Oracle(), R, Cc)
    mp = np.array(list(offset) + [0.0, 0.0, 0.0])
    zero = np.zeros(6)
    for f in range(3):
        attr = sh.SLAMAttr()
        pc0 = sh.cloud(frames[0])
        sh.L.init_slam(C.byref(attr), Pos.of(mp), C.byref(pc0))
        s.init(mp, frames[0])
        meas = sh.L.slam_localization(C.byref(attr), C.byref(sh.cloud(frames[f])),
                                      Pos.of(zero), Pos.of(zero))
        om, iters, ncp = s.localization(frames[f], zero, zero)
        q, cp, it = sh.last_frame_stats()
        assert cp == ncp
        assert np.isfinite(attr.error) and attr.error >= 0.0
        assert abs(attr.error - s.error) <= 1e-9 * max(1.0, s.error), (attr.error, s.error)
        np.testing.assert_allclose(np.array(meas.tolist()), om, rtol=0, atol=1e-6)
        if f == 0 and offset == (0.0, 0.0, 0.0):
            assert attr.error == 0.0 == s.error


def test_shim_kdtree_api_matches_reference_golden(golden):
    from shimlib import KDNode, Point, Shim, preorder
    sh = Shim(8, 8)
    for pts, perm, q, nn, nnd in _golden_sets(golden("kdtree")):
        n = len(pts)
        arr = (Point * max(n, 1))()
        if n:
            C.memmove(arr, np.ascontiguousarray(pts).ctypes.data, n * 24)
        root = sh.L.buildKDTree(arr, n, 0)
        got = np.frombuffer(bytes(arr), np.float64).reshape(-1, 3)[:n]
        _eq(got, perm, "in-place permutation")
        for i in range(len(q)):
            t = Point(*q[i])
            res = Point(np.nan, np.nan, np.nan)
            bd = C.c_double(np.inf)
            sh.L.nearestNeighborSearch(root, C.byref(t), C.byref(res), C.byref(bd), 0)
            if n:
                assert bd.value == nnd[i]
                _eq(np.array([res.x, res.y, res.z]), nn[i], "nearest")
        sh.L.freeKDTree(root)


# ------------------------------------------------- measured HBM ceiling
def test_stream_copy_copies_every_byte(gpu):
    """navgpu_stream_copy_dev (the bench's STREAM-copy ceiling) moves the
    buffer exactly, including a tail that is not a whole block's span."""
    import torch
    dev = torch.device("cuda", 0)
    n = (1 << 20) * 16 + 16 * 37
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
    dst = torch.zeros(n + 16, dtype=torch.uint8, device=dev)
    gpu.stream_copy_dev(dst, src, n)
    torch.cuda.synchronize()
    assert torch.equal(dst[:n], src)
    assert int(dst[n:].sum()) == 0


def test_two_contexts_in_flight_match_one_at_a_time():
    """bench.py's K3 step keeps two pairs in flight on two contexts (own
    stream, workspace and outputs each). Their results must equal those of
    the same pairs run one at a time: no state is shared between contexts."""
    import torch
    from navslam.gpu import NavGpu
    from navslam.synth import uniform_pair
    dev = torch.device("cuda", 0)
    R, Cc, k = 128, 1024, 8
    N = R * Cc
    pairs = [tuple(torch.from_numpy(a).to(dev) for a in uniform_pair(R, Cc, seed_src=50 + j,
                                                                     seed_tgt=60 + j))
             for j in range(4)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    ctxs = [NavGpu(0, s.cuda_stream) for s in streams]

    def outs():
        return (torch.empty((R, Cc), dtype=torch.int32, device=dev),
                torch.empty((R, Cc), dtype=torch.int32, device=dev),
                torch.empty((N, k), dtype=torch.int32, device=dev),
                torch.empty((N, k), dtype=torch.float64, device=dev))
    ref = []
    for s, t in pairs:  # one at a time
        o = outs()
        ctxs[0].pair_knn_dev(s, t, R, Cc, k, *o)
        torch.cuda.synchronize()
        ref.append([x.cpu().numpy() for x in o])
    got = [outs() for _ in pairs]
    for j, (s, t) in enumerate(pairs):  # two in flight
        ctxs[j % 2].pair_knn_dev(s, t, R, Cc, k, *got[j])
    torch.cuda.synchronize()
    for j in range(len(pairs)):
        for a, b, what in zip(got[j], ref[j], ("src_mask", "tgt_mask", "idx", "dist")):
            _eq(a.cpu().numpy(), b, f"pair {j} {what}")
    for c in ctxs:
        c.close()


def test_pair_knn_on_l9_scans_vs_oracle(kgpu, orc):
    """The bench's pair entry point (navgpu_pair_knn_dev: curvature of both
    clouds on a side stream + global k-NN) on lidar-shaped scans: masks
    against the oracle's extract_feature (src/slam.c:11-61) and every query
    against its exact grid k-NN."""
    import torch
    from navslam.synth import l9_pair
    dev = torch.device("cuda", 0)
    R, Cc, k = 64, 2048, 8
    src, tgt = l9_pair(R, Cc, seed=23)
    s, t = torch.from_numpy(src).to(dev), torch.from_numpy(tgt).to(dev)
    sm = torch.empty((R, Cc), dtype=torch.int32, device=dev)
    tm = torch.empty((R, Cc), dtype=torch.int32, device=dev)
    idx = torch.empty((R * Cc, k), dtype=torch.int32, device=dev)
    dst = torch.empty((R * Cc, k), dtype=torch.float64, device=dev)
    kgpu.pair_knn_dev(s, t, R, Cc, k, sm, tm, idx, dst)
    torch.cuda.synchronize()
    kgpu.knn_check()
    _eq(sm.cpu().numpy(), orc.extract_feature(src), "src mask")
    _eq(tm.cpu().numpy(), orc.extract_feature(tgt), "tgt mask")
    ri, rd = _memo("pair_l9", lambda: orc.knn_grid(tgt, src, k))
    _eq(idx.cpu().numpy(), ri, "idx")
    _eq(dst.cpu().numpy(), rd, "dist")


def _k5_trace():
    """tests/golden/k5_trace.npz (make_k5_trace.py): the pinned oracle's pose
    trace of the bench's K5 stream (rank 0: 128 x 2048, 8 frames, seed 11)."""
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "k5_trace.npz")
    with np.load(path) as z:
        return {k: z[k] for k in z.files}


def _k5_run(monkeypatch, n, adam, trees="1"):
    """The bench's K5 loop (bench.py run_k5, src/main.c:361-431) through the
    drop-in shim for n frames: per-frame pose, error and correspondences."""
    monkeypatch.setenv("NAVSLAM_QUIET", "1")
    monkeypatch.setenv("NAVSLAM_HOST_TREES", trees)
    if adam == "fast":
        monkeypatch.setenv("NAVSLAM_ADAM", "fast")
    else:
        monkeypatch.delenv("NAVSLAM_ADAM", raising=False)
    from shimlib import Pos, Shim
    from navslam.synth import l9_stream, l9_stream_index
    tr = _k5_trace()
    R, Cc, F, seed = (int(tr[k]) for k in ("R", "C", "F", "seed"))
    frames = l9_stream(R, Cc, F, seed=seed)
    sh = Shim(R, Cc)
    attr = sh.SLAMAttr()
    pcs = [sh.cloud(frames[f], ts=f) for f in range(F)]
    zero = Pos.of([0.0] * 6)
    sh.L.init_slam(C.byref(attr), zero, C.byref(pcs[0]))
    last = zero
    pose, err, corr = [], [], []
    for i in range(1, n + 1):
        pc = pcs[l9_stream_index(i, F)]
        meas = sh.L.slam_localization(C.byref(attr), C.byref(pc), last, last)
        sh.L.slam_mapping(C.byref(attr), meas, C.byref(pc))
        pose.append(meas.tolist())
        err.append(attr.error)
        corr.append(sh.last_frame_stats()[1])
        last = meas
    return tr, np.array(pose), np.array(err), np.array(corr)


@pytest.mark.parametrize("trees", ["1", "0"])
def test_k5_exact_stream_matches_trace_bit_exact(monkeypatch, trees):
    """K5 exact mode (the default: the reference's sequential dedup + Adam
    sums on the host, ~30 ms per frame) over the first 200 frames of the
    bench's stream (25 back-and-forth passes over its 8 frames, the map ring
    wrapped twice): every pose, error and correspondence count bit-exact
    against the committed oracle trace, host trees on and off (lazy rows)."""
    n = 200
    tr, pose, err, corr = _k5_run(monkeypatch, n, "exact", trees)
    _eq(pose, tr["pose"][:n], "K5 exact poses vs trace")
    _eq(err, tr["error"][:n], "K5 exact errors vs trace")
    _eq(corr, tr["corr"][:n], "K5 exact correspondences vs trace")


@pytest.mark.parametrize("trees", ["1", "0"])
def test_k5_fast_stream_vs_trace(monkeypatch, trees):
    """K5 fast mode (GPU dedup + closed-form Adam sums, NAVSLAM_ADAM=fast)
    running freely over the whole configured stream, every frame the trace
    holds (10,000: BASELINE.json configs[4]; 714 back-and-forth passes over
    the 8 ray-cast frames, under a millisecond each): the pose chain against
    the committed oracle trace. The order-free sums round differently from
    the reference's sequential ones, so the bound is on the
    drift: translation RMSE over all frames <= 1e-6 mm and every coordinate
    within 1e-5 (mm or degrees); the correspondence count of every frame
    equal."""
    n = len(_k5_trace()["pose"])
    tr, pose, err, corr = _k5_run(monkeypatch, n, "fast", trees)
    ref = tr["pose"][:n]
    d = pose[:, :3] - ref[:, :3]
    rmse = float(np.sqrt(np.mean(np.sum(d * d, axis=1))))
    assert rmse <= 1e-6, rmse
    np.testing.assert_allclose(pose, ref, rtol=0, atol=1e-5)
    _eq(corr, tr["corr"][:n], "K5 fast correspondences vs trace")
