#!/usr/bin/env python3
"""Scan-pair matches/sec on MI355X (BASELINE.json metric), one process per GPU.

Default workload (K3, BASELINE.json configs[2] — the config the metric is
quoted on, "1M-pt clouds"): one scan pair per GPU, 1,048,576 points per cloud
arranged as a 512x2048 grid, x,y,z ~ U[0,1000) mm. One step = the whole
front end on that pair, inputs already resident in HBM:
    curvature/features of source and target (R1)
  + index build over the target (radix-binned uniform grid)
  + exact k=8 nearest neighbours of every source point.
value = matches (query points matched) over all ranks / max-over-ranks time.

`--workload k2` runs the per-row slam.c mode instead (128x2048 L9-shaped
pair, 1-NN, exact reference KD semantics), `--workload k4` a batch of
256 K2 pairs sharded over the ranks with an RCCL all-gather of the match
sets (the north star's batched case), and `--workload k5` the streaming
L9 loop of src/main.c:361-431 (slam_localization + slam_mapping per frame)
through the drop-in C ABI (libnavslam_128x2048.so), one step = one frame.

K3 keeps three pairs in flight by default (--inflight): consecutive steps
alternate over three library contexts, each with its own stream, workspace
and outputs, so one pair's memory-bound index build overlaps the previous
pairs' latency-bound queries. Every step still processes one whole pair.

Launch: python bench.py [--gpus N --steps K --warmup W]. For N > 1 either
under torch.distributed.run (--nproc-per-node N, one rank per GPU, RCCL), or
plain `python bench.py --gpus N`, which starts that launcher itself as a child
process; a WORLD_SIZE that differs from --gpus is an error.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nav-slam_amd"))

import numpy as np  # noqa: E402

METRIC = ("scan-pair matches/sec (feature-extract + kNN), 1M-pt clouds, 1/2/4/8 MI355X; "
          "% HBM roofline")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (8.0 TB/s spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # (r6: 200 timed steps by default. With pairs in flight the timed region
    # starts on an empty pipeline and ends draining it; over 20 steps that
    # and the first steps' cold clocks cost the K3 line ~9 % (0.2386-0.2427
    # vs 0.2197-0.2206 ms per pair at 200, profiles/r6/k3_steps_ab.txt); a
    # K3 step is ~0.22 ms, the slowest default line (K4i) ~6 s)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", choices=["k3", "k2", "k4", "k5"], default="k3")
    p.add_argument("--stream-frames", type=int, default=8,
                   help="k5: distinct ray-cast frames, replayed back and forth")
    p.add_argument("--k5-mode", choices=["exact", "fast"], default="exact",
                   help="k5: exact = the reference's sequential dedup + Adam sums on the "
                        "host (bit-exact); fast = GPU dedup + closed-form Adam sums "
                        "(NAVSLAM_ADAM=fast, pose RMSE reported)")
    p.add_argument("--cpu-frames", type=int, default=3,
                   help="k5: frames of the CPU reference run (pose RMSE + timing)")
    p.add_argument("--k", type=int, default=8)
    p.add_argument("--rows", type=int, default=None)
    p.add_argument("--cols", type=int, default=None)
    p.add_argument("--pairs", type=int, default=256, help="k4: total pairs")
    p.add_argument("--integer-mm", action="store_true",
                   help="k2/k4: coordinates rounded to whole mm (the tie-heavy case: rows "
                        "with equidistant targets take the reference tree)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--graph", action="store_true",
                   help="k3: capture one step into a hipGraph and replay it")
    p.add_argument("--inflight", type=int, default=3,
                   help="k3: pairs in flight -- consecutive steps alternate over this many "
                        "contexts (own stream, workspace and outputs each), so one pair's "
                        "HBM-bound index build overlaps the previous pairs' latency-bound "
                        "queries (r5, k_knng: 2 -> 0.241-0.245 ms/pair, 3 -> 0.233-0.238, "
                        "4 -> 0.248-0.249; r1's kernels: 2 and 3 both 0.294); "
                        "--graph needs --inflight 1")
    p.add_argument("--no-events", action="store_true",
                   help="A/B diagnostic: no HIP timing events in the timed region (the line "
                        "then has no kernel times or roofline)")
    p.add_argument("--cpu-reps", type=int, default=5,
                   help="CPU baseline: timed repetitions (median), after one untimed warm-up")
    p.add_argument("--resident-pairs", type=int, default=9,
                   help="k3: distinct scan pairs resident in HBM, rotated step by step "
                        "(9 x 48 MiB = 432 MiB, above the 256 MiB Infinity Cache, so the "
                        "inputs of a step are not the previous step's cache hits)")
    p.add_argument("--iso-steps", type=int, default=10,
                   help="k3: extra steps on one context alone after the timed region, "
                        "for the isolated kernel durations")
    p.add_argument("--traffic-csv", default=None,
                   help="comma-separated rocprofv3 --pmc counter_collection.csv files "
                        "(FETCH_SIZE and WRITE_SIZE passes) to derive HBM bytes")
    p.add_argument("--traffic-json", default=None,
                   help="per-step HBM bytes from the PMC passes (scripts/round_evidence.sh "
                        "writes them via scripts/traffic_json.py; default "
                        "profiles/traffic_<workload>.json)")
    p.add_argument("--no-traffic-json", action="store_true")
    p.add_argument("--no-stream-copy", action="store_true",
                   help="skip the STREAM-copy ceiling measurement")
    p.add_argument("--json-out", default=None)
    p.add_argument("--dry-run", action="store_true",
                   help="rank plumbing only (no GPU): every rank joins a gloo group, takes "
                        "its K4 shard of --pairs and reports; rank 0 prints one JSON line")
    return p.parse_args()


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a):
    """`--gpus N` (N > 1) run without a launcher: start N rank processes
    through torch.distributed.run as ONE child process (one rank per GPU,
    rendezvous on 127.0.0.1) and return its exit code. Nothing here touches
    the GPU: the parent only waits (no exec from a process that initialised
    HIP)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def check_ranks(a, ws, local):
    """The rank count must be what --gpus asks for, and every rank needs its
    own visible device (torch.cuda.device_count() does not initialise HIP on
    this image). Returns an error message, or None."""
    if ws != a.gpus:
        return (f"bench.py: --gpus {a.gpus} but WORLD_SIZE={ws}; launch "
                f"`python bench.py --gpus N` (it starts the N ranks itself) or "
                f"torch.distributed.run with --nproc-per-node equal to --gpus")
    if a.dry_run:
        return None
    import torch
    nd = torch.cuda.device_count()
    if local >= nd:
        return (f"bench.py: rank with LOCAL_RANK={local} of --gpus {a.gpus}, but only {nd} "
                "device(s) visible")
    return None


def run_dry(a, ws, rank):
    """--dry-run: the K4 rank plumbing on gloo (CPU): every rank takes its
    contiguous shard of --pairs; the ranks' (rank, lo, hi) are all-gathered
    and rank 0 returns them."""
    import torch
    import torch.distributed as dist
    from navslam import shard
    if ws > 1:
        dist.init_process_group("gloo")
    lo, hi = shard.shard_pairs(a.pairs, ws, rank)
    mine = torch.tensor([rank, lo, hi], dtype=torch.int64)
    if ws > 1:
        parts = [torch.empty_like(mine) for _ in range(ws)]
        dist.all_gather(parts, mine)
    else:
        parts = [mine]
    total = shard.sum_over_ranks(hi - lo, torch.device("cpu"))
    out = None
    if rank == 0:
        out = {"dry_run": True, "n_gpus": ws, "gpus_requested": a.gpus,
               "ranks_reported": [p.tolist() for p in parts], "pairs": int(total),
               "workload": a.workload}
    if ws > 1:
        dist.destroy_process_group()
    return out


def host_info():
    """nproc, the CPU model and the threads the multi-thread legs use."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def median_after_warmup(fn, reps):
    """One untimed warm-up, then the median of `reps` timed runs."""
    fn()
    ts = []
    for _ in range(max(1, reps)):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def _ref_lib():
    import ctypes as C
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libref8x8.so")
    if not os.path.exists(ref_path):
        return None
    lib = C.CDLL(ref_path)
    lib.buildKDTree.restype = C.c_void_p
    lib.buildKDTree.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    lib.freeKDTree.argtypes = [C.c_void_p]
    return lib


def _addr(lib, name):
    import ctypes as C
    return C.cast(getattr(lib, name), C.c_void_p).value


def cpu_baseline_k3(src, tgt, k, reps):
    """The reference's own CPU path on the K3 pair (rank 0, N = 1 only):
    oracle/_ref/libref8x8.so = utils/kdtree.c compiled as-is -- buildKDTree
    over the 1M target (utils/kdtree.c:65-82) and nearestNeighborSearch for
    every source point (utils/kdtree.c:110-152; the reference has k = 1 only)
    -- plus the oracle's bit-exact restatement of extract_feature
    (src/slam.c:11-61) on both 512x2048 clouds (the reference's own is fixed
    to 8x8). Two legs, each the median of `reps` after one warm-up:
      1 core    : as the reference runs (single-threaded);
      threads_N : OpenMP over the queries on N threads (the search only reads
                  the tree) and over rows for the curvature; the tree build is
                  the reference's serial recursion. N = OMP_NUM_THREADS: the
                  GPU box allots 16 host CPUs to a one-GPU job (its harness
                  sets OMP_NUM_THREADS=16 and asks jobs to keep within it);
                  nproc counts the whole shared 8-GPU host (host_info), whose
                  other CPUs belong to other jobs.
    """
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import Oracle
    orc = Oracle()
    lib = _ref_lib()
    kind = "reference" if lib is not None else "port"
    N = src.shape[0] * src.shape[1]
    q = np.ascontiguousarray(src.reshape(-1, 3))

    def run(threads):
        def once():
            if threads == 1:
                orc.extract_feature(src)
                orc.extract_feature(tgt)
            else:
                orc.extract_feature_mt(src, threads)
                orc.extract_feature_mt(tgt, threads)
            if lib is not None:
                arr = np.ascontiguousarray(tgt.reshape(-1, 3)).copy()
                root = lib.buildKDTree(arr.ctypes.data, N, 0)
                fn = _addr(lib, "nearestNeighborSearch")
                (orc.ref_nn_batch if threads == 1 else orc.ref_nn_batch_mt)(fn, root, q)
                lib.freeKDTree(root)
            else:
                t, _ = orc.kd_build(tgt.reshape(-1, 3))
                orc.kd_nn_batch(t, q)
        return once

    host = host_info()
    t1, ts1 = median_after_warmup(run(1), reps)
    threads = orc.max_threads()
    tall, tsall = median_after_warmup(run(threads), reps)
    return {"value": round(N / t1, 1), "unit": "matches/s", "cores": 1, "kind": kind,
            "seconds_per_pair": round(t1, 4), "runs_s": [round(t, 4) for t in ts1],
            f"threads_{threads}": {"value": round(N / tall, 1), "unit": "matches/s",
                                   "cores": threads, "seconds_per_pair": round(tall, 4),
                                   "runs_s": [round(t, 4) for t in tsall],
                                   "note": "OpenMP over queries and curvature rows; serial "
                                           "tree build; N = OMP_NUM_THREADS, the host CPUs the "
                                           "GPU box allots to a one-GPU job (nproc counts the "
                                           "whole shared host)"},
            "host": host,
            "sample": (f"the full K3 pair 0 ({N} queries vs {N} targets), median of {reps} after "
                       "1 warm-up: extract_feature on both clouds + buildKDTree + "
                       "nearestNeighborSearch per source point, k=1 (the reference has no "
                       "k-NN; k=8 would cost more)")}


def cpu_baseline_k2(src, tgt, reps):
    """The reference's CPU path for one per-row (slam.c) pair, rank 0 only:
    extract_feature on both clouds (the oracle's bit-exact restatement; the
    reference's is fixed to 8x8) + for every row the reference's own
    buildKDTree over the target row's features and nearestNeighborSearch for
    each source feature (oracle/_ref = utils/kdtree.c compiled as-is), which
    is what src/slam.c:162-172,230-244 runs per frame. 1 core (as the
    reference) and N threads (OpenMP over rows, N = OMP_NUM_THREADS); median of `reps` after one
    warm-up."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import Oracle
    orc = Oracle()
    lib = _ref_lib()
    if lib is None:
        return None
    fns = tuple(_addr(lib, f) for f in ("buildKDTree", "nearestNeighborSearch", "freeKDTree"))
    nq = [0]

    def run(threads):
        def once():
            if threads == 1:
                sm, tm = orc.extract_feature(src), orc.extract_feature(tgt)
            else:
                sm, tm = orc.extract_feature_mt(src, threads), orc.extract_feature_mt(tgt, threads)
            nq[0] = orc.ref_rows_match(fns, src, tgt, sm, tm, threads)[2]
        return once

    t1, ts1 = median_after_warmup(run(1), reps)
    threads = orc.max_threads()
    tall, tsall = median_after_warmup(run(threads), reps)
    return {"value": round(nq[0] / t1, 1), "unit": "matches/s", "cores": 1, "kind": "reference",
            "seconds_per_pair": round(t1, 5), "runs_s": [round(t, 5) for t in ts1],
            f"threads_{threads}": {"value": round(nq[0] / tall, 1), "unit": "matches/s",
                                   "cores": threads, "seconds_per_pair": round(tall, 5),
                                   "runs_s": [round(t, 5) for t in tsall],
                                   "note": "OpenMP over rows (build + queries) and curvature "
                                           "rows; N = OMP_NUM_THREADS, the host CPUs the GPU box "
                                           "allots to a one-GPU job"},
            "host": host_info(),
            "sample": (f"one {src.shape[0]}x{src.shape[1]} L9-shaped pair ({nq[0]} source-feature "
                       f"queries), median of {reps} after 1 warm-up: extract_feature x2 + per-row "
                       "buildKDTree + nearestNeighborSearch per source feature")}


def run_k5(a, ws, rank, dev):
    """K5 (BASELINE.json configs[4]): the L9 streaming loop of
    src/main.c:361-431 through the drop-in ABI -- init_slam on frame 0, then per
    frame slam_localization(frame, last, last) + slam_mapping(measured). Every
    frame rebuilds the target (per-row trees of the new frame's features in
    the global frame) on the GPU; dedup and the 3-DOF Adam run on the host,
    bit-exact (their sequential f64 sums fix the rounding order). Host
    pointers in and out, as the reference API has them: the per-frame PCIe
    copies are inside the timed region. Replicas only (a pose chain does not
    shard): each rank runs its own stream."""
    import torch
    import torch.distributed as dist
    from navslam import shard, synth
    from navslam.abi import Pos, Shim
    os.environ.setdefault("NAVSLAM_QUIET", "1")   # no per-iteration printf
    if a.k5_mode == "fast":
        os.environ["NAVSLAM_ADAM"] = "fast"
    else:
        os.environ.pop("NAVSLAM_ADAM", None)
    os.environ.setdefault("NAVSLAM_DEVICE", str(dev.index))
    R, Cc = a.rows or 128, a.cols or 2048
    F = max(1, a.stream_frames)
    frames = synth.l9_stream(R, Cc, F, seed=11 + rank)
    sh = Shim(R, Cc)
    pcs = [sh.cloud(frames[f], ts=f) for f in range(F)]
    attr = sh.SLAMAttr()
    # the caller's SLAM_attr (100 map slots, 630 MB at 128 x 2048) touched once
    # before timing: a long run writes every slot many times, so a short
    # timed run must not pay the first-touch page faults of 60 fresh slots
    import ctypes
    ctypes.memset(ctypes.addressof(attr), 0, ctypes.sizeof(attr))
    zero = Pos.of([0.0] * 6)
    sh.L.init_slam(attr, zero, pcs[0])
    poses, state = [], {"i": 0, "last": zero, "q": 0}

    # kernel timing (HIP events) on every 4th frame of the timed region only:
    # events on every frame cost the frame ~4 % (r5)
    ev = {"ctx": None, "L": None, "on": False}

    def frame():
        state["i"] += 1
        if ev["on"]:
            ev["L"].navgpu_timing_enable(ev["ctx"], 1 if state["i"] % 4 == 0 else 0)
        pc = pcs[synth.l9_stream_index(state["i"], F)]
        last = state["last"]
        meas = sh.L.slam_localization(attr, pc, last, last)
        sh.L.slam_mapping(attr, meas, pc)
        state["last"] = meas
        state["q"] += sh.last_frame_stats()[0]
        poses.append(meas.tolist())

    for _ in range(a.warmup):
        frame()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    ctx = sh.context()
    from navslam.gpu import load_library
    L = load_library()
    ev.update(ctx=ctx, L=L, on=not a.no_events)
    names = ["rows_build", "rows_query", "rows_retree"] + (["rows_corr"] if a.k5_mode == "fast" else [])
    for n in names:
        L.navgpu_timing_read(ctx, n.encode(), 1)
    q0 = state["q"]
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        frame()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    t1 = time.perf_counter()
    ev["on"] = False
    L.navgpu_timing_enable(ctx, 0)
    kt = {}
    for n in names:
        cnt = L.navgpu_timing_count(ctx, n.encode())
        kt[n] = (L.navgpu_timing_read(ctx, n.encode(), 1), cnt)
    elapsed = shard.max_over_ranks(t1 - t0, dev)
    matches = shard.sum_over_ranks(state["q"] - q0, dev)
    frames_all = shard.sum_over_ranks(a.steps, dev)
    if rank != 0:
        return None
    floor = k5_copy_floor(L, ctx, pcs, attr, R * Cc)
    cpu = None
    if not a.no_cpu_baseline and a.cpu_frames > 0:
        cpu = cpu_baseline_k5(frames, F, min(a.cpu_frames, len(poses)), poses)
    vs_trace = k5_vs_trace(poses, frames, R, Cc, F, 11 + rank, a.warmup)
    # (a region never entered this run, e.g. rows_retree with host trees on,
    # reads as count 0)
    per_frame = lambda n: 1000.0 * kt[n][0] / kt[n][1] if kt[n][1] > 0 else 0.0
    gpu_us = sum(per_frame(n) for n in names)
    # SURVEY 8(d) bytes per frame, per-row mode: build reads 24 B per target
    # feature point + the query stage 24 B per query + 24 B per target
    # feature + 12 B per match (k = 1): with T ~ Q ~ queries per frame
    qpf = (state["q"] - q0) / max(a.steps, 1)
    bytes_pf = int(24 * qpf + (24 + 24 + 12) * qpf)
    ach = bytes_pf / (gpu_us * 1e-6) / 1e9 if gpu_us > 0 else None
    tj = load_traffic(a, {"workload": traffic_tag(a), "points_per_cloud": R * Cc})
    roof = {"bound": "hbm", "achieved": round(ach, 2) if ach else None, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 6) if ach else None,
            "traffic": tj and tj.get("bytes_per_step"),
            "kernel": "k_rows_build + k_rows_query (+ k_rows_retree, k_rows_corr) per frame",
            "avg_us": round(gpu_us, 2), "bytes_per_launch": bytes_pf,
            "bytes_model": "24 B/target feature (build) + 24 Q + 24 T + 12 Q (query), SURVEY 8d",
            "note": ("latency-bound per-row kernels; " + ("a frame is host-bound (sequential "
                     "Adam sums)" if a.k5_mode == "exact" else "frames carry the API's host "
                     "copies (global map slot, host trees)"))}
    out = {"metric": METRIC, "value": round(matches / elapsed, 1), "unit": "matches/s",
           "n_gpus": ws, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": round(1000.0 * elapsed / a.steps, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": (f"synthetic L9 stream: {F} ray-cast {R}x{Cc} frames along a walk "
                    "(navslam.synth.l9_stream), replayed back and forth"),
           "config": {"workload": (f"K5: streaming L9 loop (src/main.c:361-431) through the "
                                   f"drop-in ABI, {R}x{Cc} frames, per-frame target rebuild, "
                                   + ("bit-exact host dedup + Adam" if a.k5_mode == "exact" else
                                      "GPU dedup + closed-form Adam sums (NAVSLAM_ADAM=fast)")),
                      "k5_mode": a.k5_mode,
                      # NAVSLAM_HOST_TREES=0: no KDNode trees handed to the
                      # caller, row trees built only for rows with a tie (r4)
                      "host_trees": os.environ.get("NAVSLAM_HOST_TREES", "1") != "0",
                      "parallelism": f"replicas x{ws}", "points_per_frame": R * Cc,
                      "frames_per_s": round(frames_all / elapsed, 2),
                      "queries_per_frame": round(qpf, 1), "mode": "rows"},
           "roofline": roof, "curvature_plus_query": None,
           "kernel_us": {n: round(per_frame(n), 2) for n in names},
           # the frame's API copies alone (the same pageable frame and map-slot
           # buffers, the same entry points, nothing else on the device): the
           # floor a frame of this API cannot go below
           "copy_floor_ms": round(floor["ms"], 4),
           "copy_floor": floor,
           "frac_of_copy_floor": round(floor["ms"] / (1000.0 * elapsed / a.steps), 4),
           "pose_vs_trace": vs_trace,
           "cpu_baseline": cpu}
    return out


def k5_vs_trace(poses, frames, R, Cc, F, seed, warmup):
    """The run's pose chain against the committed oracle trace of the same
    stream (tests/golden/k5_trace.npz, make_k5_trace.py): every frame the
    trace covers, warmup and timed alike (frame i's pose is poses[i - 1]).
    None when this rank's stream is not the trace's."""
    import hashlib
    path = os.path.join(ROOT, "tests", "golden", "k5_trace.npz")
    if not os.path.exists(path):
        return None
    with np.load(path) as z:
        tr = {k: z[k] for k in z.files}
    if (int(tr["R"]), int(tr["C"]), int(tr["F"]), int(tr["seed"])) != (R, Cc, F, seed):
        return None
    if hashlib.sha256(np.ascontiguousarray(frames, np.float64).tobytes()).hexdigest() != \
            str(tr["frames_sha256"]):
        return None
    n = min(len(poses), len(tr["pose"]))
    g, c = np.asarray(poses[:n]), tr["pose"][:n]
    d = g[:, :3] - c[:, :3]
    timed = slice(warmup, n)
    return {"frames": n, "timed_frames": max(0, n - warmup),
            "rmse_mm": float(np.sqrt(np.mean(np.sum(d * d, axis=1)))),
            "rmse_mm_timed": (float(np.sqrt(np.mean(np.sum(d[timed] ** 2, axis=1))))
                              if n > warmup else None),
            "max_abs_mm_or_deg": float(np.max(np.abs(g - c))),
            "bit_exact": bool(np.array_equal(g, c)),
            "source": "tests/golden/k5_trace.npz (the pinned oracle's src/slam.c restatement, "
                      f"{len(tr['pose'])} frames)"}


def k5_copy_floor(L, ctx, pcs, attr, npts, reps=20):
    """Per-frame floor of the K5 API's host copies: the frame uploaded twice
    (slam_localization and slam_mapping each upload their lidar cloud) and
    the 24 B/point map slot downloaded once, timed alone over `reps` frames
    with the same pageable buffers and navgpu_upload/download."""
    import ctypes
    nb = 24 * npts
    d = ctypes.c_void_p()
    if L.navgpu_malloc(ctx, nb, ctypes.byref(d)) != 0:
        raise RuntimeError("k5_copy_floor: device allocation failed")
    try:
        src = ctypes.addressof(pcs[0].pos)
        dst = ctypes.addressof(attr.globalPointCloud[0].pos)
        t = {"h2d": 0.0, "d2h": 0.0}
        for rep in range(reps + 2):  # two warm-up frames
            a0 = time.perf_counter()
            for _ in range(2):
                L.navgpu_upload(ctx, d, src, nb)
            L.navgpu_sync(ctx)
            a1 = time.perf_counter()
            L.navgpu_download(ctx, dst, d, nb)
            L.navgpu_sync(ctx)
            a2 = time.perf_counter()
            if rep >= 2:
                t["h2d"] += a1 - a0
                t["d2h"] += a2 - a1
    finally:
        L.navgpu_free(ctx, d)
    h2d, d2h = 1000.0 * t["h2d"] / reps, 1000.0 * t["d2h"] / reps
    return {"ms": h2d + d2h, "h2d_ms_2x": round(h2d, 4), "d2h_ms": round(d2h, 4),
            "bytes": 3 * nb, "gbs": round(3 * nb / ((h2d + d2h) * 1e-3) / 1e9, 2),
            "buffers": "pageable (the frame's PointCloud, the map slot)"}


def cpu_baseline_k5(frames, F, nf, gpu_poses):
    """The same stream's first `nf` frames through the oracle's restatement of
    src/slam.c (single-threaded; the reference's own build is fixed to 8x8,
    utils/pointcloud.h:9-10): seconds per frame, and the pose RMSE of the
    GPU run against it over those frames."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import Oracle, OracleSlam
    from navslam import synth
    orc = Oracle()
    R, Cc = frames.shape[1], frames.shape[2]
    s = OracleSlam(orc, R, Cc)
    z = np.zeros(6)
    s.init(z, frames[0])
    last, poses, ts = z, [], []
    for i in range(1, nf + 1):
        f = frames[synth.l9_stream_index(i, F)]
        t0 = time.perf_counter()
        meas, _, _ = s.localization(f, last, last)
        s.mapping(meas, f)
        ts.append(time.perf_counter() - t0)
        poses.append(meas)
        last = meas
    g = np.asarray(gpu_poses[:nf])[:, :3]
    c = np.asarray(poses)[:, :3]
    rmse = float(np.sqrt(np.mean(np.sum((g - c) ** 2, axis=1))))
    exact = bool(np.array_equal(np.asarray(gpu_poses[:nf]), np.asarray(poses)))
    t = float(np.median(ts))
    return {"value": None, "unit": "s/frame", "seconds_per_frame": t,
            "frames_per_s": 1.0 / t, "cores": 1, "kind": "port",
            "pose_rmse_mm": rmse, "pose_bit_exact": exact,
            "sample": (f"the first {nf} frames of the same stream through the oracle's "
                       "restatement of src/slam.c at this grid (pinned bit-exact to the "
                       "reference build by tests/golden), median frame time")}


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    ws, rank, local = dist_env()
    err = check_ranks(a, ws, local)
    if err is not None:
        print(err, file=sys.stderr, flush=True)
        sys.exit(2)
    if a.dry_run:
        out = run_dry(a, ws, rank)
        if out is not None:
            print(json.dumps(out), flush=True)
        return out
    if a.workload == "k5":
        import torch
        import torch.distributed as dist
        if ws > 1:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local if ws > 1 else 0)
        torch.cuda.set_device(dev)
        out = run_k5(a, ws, rank, dev)
        if out is not None:
            line = json.dumps(out)
            print(line, flush=True)
            if a.json_out:
                with open(a.json_out, "w") as f:
                    f.write(line + "\n")
        if ws > 1:
            dist.destroy_process_group()
        return out
    import torch
    import torch.distributed as dist
    if ws > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if ws > 1 else 0)
    torch.cuda.set_device(dev)
    from navslam import shard, synth
    from navslam.gpu import NavGpu

    # the library runs on a dedicated torch stream (capturable, and the one
    # torch.cuda.synchronize() covers like any other)
    stream = torch.cuda.Stream(dev)
    g = NavGpu(dev.index, stream.cuda_stream)

    if a.workload == "k3":
        R = a.rows or 512
        Cc = a.cols or 2048
        N = R * Cc
        # distinct pairs resident in HBM, rotated per step: pair j of rank r
        # has seeds (1 + 2r + 1000 j, 2 + 2r + 1000 j); pair 0 is the
        # canonical K3 pair (seeds 1, 2 on rank 0)
        npairs = max(1, a.resident_pairs)
        s_seed, t_seed = shard.pair_seeds(rank)
        pairs_h = [synth.uniform_pair(R, Cc, seed_src=s_seed + 1000 * j,
                                      seed_tgt=t_seed + 1000 * j) for j in range(npairs)]
        src_h, tgt_h = pairs_h[0]
        pairs_d = [(torch.from_numpy(sh).to(dev), torch.from_numpy(th).to(dev))
                   for sh, th in pairs_h]
        del pairs_h
        nf = max(1, a.inflight)
        # pairs in flight: context j (its own stream, workspace and outputs)
        # takes steps j, j + nf, ...
        extra = [NavGpu(dev.index, torch.cuda.Stream(dev).cuda_stream) for _ in range(nf - 1)]
        outs = [tuple(torch.empty(shape, dtype=dt, device=dev) for shape, dt in
                      (((R, Cc), torch.int32), ((R, Cc), torch.int32), ((N, a.k), torch.int32),
                       ((N, a.k), torch.float64)))
                for _ in range(nf)]
        ctxs = [g] + extra
        turn = [0]

        def step():
            i = turn[0]
            turn[0] += 1
            src, tgt = pairs_d[i % npairs]
            ctxs[i % nf].pair_knn_dev(src, tgt, R, Cc, a.k, *outs[i % nf])

        def iso_step():  # one context alone: nothing else shares the chip
            src, tgt = pairs_d[turn[0] % npairs]
            turn[0] += 1
            g.pair_knn_dev(src, tgt, R, Cc, a.k, *outs[0])
        if a.graph and nf == 1:
            for _ in range(2):  # warm: workspace grown, nothing allocates while capturing
                step()
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                g.pair_knn_dev(pairs_d[0][0], pairs_d[0][1], R, Cc, a.k, *outs[0])
            step = graph.replay  # noqa: F811
        matches_per_step = N
        dom = "knn_query"
        dom_bytes = (24 + 24 + 12 * a.k) * N        # 24Q + 24T + 12kQ
        path_bytes = 2 * 28 * N + dom_bytes          # + curvature 28 B/pt, both clouds
        path_kernels = ["curvature", "knn_query"]
        workload = (f"K3: {N}-point scan pair ({R}x{Cc} grid, U[0,1000)^3 mm), curvature "
                    f"on both clouds + grid index build + exact k={a.k} NN of every source "
                    "point, global mode")
        data = (f"synthetic: x,y,z ~ U[0,1000) mm, numpy PCG64 seeds (1+2r+1000j, 2+2r+1000j) "
                f"on rank r, {npairs} distinct pairs j resident and rotated per step")
        # under --graph the captured step replays one resident pair
        res_pairs = 1 if (a.graph and nf == 1) else npairs
        if res_pairs == 1:
            data = data.replace(f"{npairs} distinct pairs j resident and rotated per step",
                                "one resident pair replayed by a hipGraph")
        cfg_extra = {"points_per_cloud": N, "k": a.k, "pairs_per_gpu": 1, "mode": "global",
                     "knn_mode": knn_mode(), "query_kernel": knn_query_kernel(),
                     "pairs_in_flight": nf, "resident_pairs": res_pairs,
                     "resident_bytes": res_pairs * 2 * 24 * N}
    else:
        ctxs, iso_step, nf = [g], None, 1
        R = a.rows or 128
        Cc = a.cols or 2048
        N = R * Cc
        if a.workload == "k2":
            lo, hi, pmax = 0, 1, 1
        else:  # contiguous block of the batch per rank
            lo, hi = shard.shard_pairs(a.pairs, ws, rank)
            pmax = -(-a.pairs // ws)
        pairs = hi - lo
        srcs, tgts = [], []
        for p in range(lo, hi):
            s_h, t_h = synth.l9_pair(R, Cc, seed=p + 5, integer_mm=a.integer_mm)
            srcs.append(torch.from_numpy(s_h).to(dev))
            tgts.append(torch.from_numpy(t_h).to(dev))
            if a.workload == "k4" and p - lo >= 7:   # 8 distinct pairs, cycled
                break
        nd = len(srcs)
        if a.workload == "k4" and pairs:  # the rank's batch, resident as [pairs][R][C]
            bsrc = torch.stack([srcs[p % nd] for p in range(pairs)])
            btgt = torch.stack([tgts[p % nd] for p in range(pairs)])
        sm = torch.empty((pmax, R, Cc), dtype=torch.int32, device=dev)
        tm = torch.empty((pmax, R, Cc), dtype=torch.int32, device=dev)
        # the rank's match sets as ONE packed buffer: idx [pmax][R][C] int32,
        # then dist [pmax][R][C] f64 -- 12 B per grid cell, so the
        # K4 exchange is a single all-gather
        packed = torch.empty(pmax * N * 12, dtype=torch.uint8, device=dev)
        idx, dst = shard.match_views(packed, pmax, R, Cc)
        idx.fill_(-1)
        gather_buf = None
        if a.workload == "k4" and ws > 1:
            gather_buf = torch.empty(ws * packed.numel(), dtype=torch.uint8, device=dev)
        do_gather = [True]  # scans/s are also reported without the gather

        def step():
            if a.workload == "k4":  # one launch over the rank's whole batch
                if pairs:
                    g.rows_match_batch_dev(bsrc, btgt, pairs, R, Cc, sm, tm, idx, dst)
            else:
                g.rows_match_dev(srcs[0], tgts[0], R, Cc, sm[0], tm[0], idx[0], dst[0])
            if gather_buf is not None and do_gather[0]:
                shard.gather_matches(packed, gather_buf)
        # matches = feature queries actually searched (constant per pair)
        step()
        torch.cuda.synchronize()
        tie_rows = g.rows_tie_rows()  # rows that needed the reference tree
        matches_per_step = 0
        if pairs:
            matches_per_step = int((sm[:nd] == 1).sum().item()) * (pairs // nd) \
                + int((sm[: pairs % nd] == 1).sum().item())
        dom = "rows_match"
        # curvature 28 B per grid point of both clouds + the
        # query stage 24 B per query + 24 B per target feature + 12 B per
        # match (k = 1), over the pairs one launch processes
        nmp = min(pairs, nd) if pairs else 0
        feat_t = int((tm[:nmp] == 1).sum().item()) if nmp else 0
        per_pair = (2 * 28 * N + 36 * (matches_per_step / max(pairs, 1))
                    + 24 * feat_t / max(nmp, 1)) if pairs else 0
        dom_bytes = int(per_pair * pairs) if pairs else None
        path_bytes = None
        path_kernels = ["rows_match"]
        workload = (f"{'K2' if a.workload == 'k2' else 'K4'}: {pairs} L9-shaped {R}x{Cc} "
                    "scan pair(s) per GPU, per-row mode (slam.c semantics): curvature of both "
                    "clouds + exact 1-NN of every source feature against its target row (the "
                    "reference KD semantics; its tree built only for rows with a distance tie)"
                    + (", RCCL all-gather of the match sets (idx + dist, 12 B per cell)"
                       if gather_buf is not None else ""))
        data = ("synthetic L9-shaped range images (navslam.synth.l9_pair), fixed seeds"
                + (", coordinates rounded to whole mm" if a.integer_mm else ""))
        cfg_extra = {"points_per_cloud": N, "k": 1, "pairs_per_gpu": pairs, "mode": "rows",
                     "integer_mm": bool(a.integer_mm), "tie_rows": tie_rows,
                     "rows_per_step": pairs * R}

    # setup: every context of the pairs in flight allocates its workspace on
    # its first call, so each makes one call here, whatever --warmup is
    # (outside the warmup and timed steps; the rotation is restarted)
    if a.workload == "k3" and nf > 1:
        for _ in range(nf):
            step()
        turn[0] = 0
    # warmup (grows the workspace, JITs nothing)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    # kernel timing on every context; each kernel's average is its summed
    # time over its own launch count (with pairs in flight, a context runs
    # only every nf-th step). With pairs in flight the timed region records
    # only the dominant query stage: events around every region of every
    # step cost the K3 step ~2 % (r5: 0.2443 vs 0.2386 ms with no events,
    # three interleaved rounds); the build and curvature come from the
    # isolated steps after it
    names = sorted(set(path_kernels + [dom] + (["knn_build"] if a.workload == "k3" else [])))
    only_dom = a.workload == "k3" and nf > 1

    def timing_on(on):
        for c in ctxs:
            c.timing(on)
            c.timing_select(dom if (on and only_dom) else None)
            for name in names:
                c.timing_read(name, reset=True)

    def timing_collect():
        agg = {}
        for name in names:
            ms = n = 0
            for c in ctxs:
                m_, n_ = c.timing_read(name, reset=True)
                if n_ > 0 and m_ >= 0:  # (-1 ms: the region was never recorded here)
                    ms += m_
                    n += n_
            agg[name] = (ms, n)
        return agg
    timing_on(not a.no_events)
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if ws > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = shard.max_over_ranks(t1 - t0, dev)
    job_matches = shard.sum_over_ranks(matches_per_step, dev)
    kt = timing_collect()
    # isolated kernel durations: the same steps on one context alone, after
    # the timed region (K3 with pairs in flight only)
    kt_iso = None
    if iso_step is not None and nf > 1 and a.iso_steps > 0:
        g.timing_select(None)  # every region of the isolated steps
        for _ in range(a.iso_steps):
            iso_step()
        torch.cuda.synchronize()
        kt_iso = timing_collect()
    timing_on(False)
    # K4 on N > 1 ranks: the same steps again without the all-gather
    no_gather = None
    if a.workload in ("k2", "k4") and gather_buf is not None:
        do_gather[0] = False
        torch.cuda.synchronize()
        dist.barrier()
        t2 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        dist.barrier()
        el2 = shard.max_over_ranks(time.perf_counter() - t2, dev)
        do_gather[0] = True
        no_gather = {"value": round(job_matches * a.steps / el2, 1),
                     "ms_per_step": round(1000.0 * el2 / a.steps, 4),
                     "gather_bytes_per_rank": int(ws * packed.numel())}
    # measured HBM ceiling: a STREAM copy of 1 GiB, far above the
    # 256 MiB Infinity Cache, on the library's stream (read + write bytes)
    stream_copy = None
    if rank == 0 and not a.no_stream_copy:
        nb = 1 << 30
        sbuf = torch.empty(nb, dtype=torch.uint8, device=dev)
        dbuf = torch.empty(nb, dtype=torch.uint8, device=dev)
        sbuf.fill_(1)
        for _ in range(3):
            g.stream_copy_dev(dbuf, sbuf, nb)
        torch.cuda.synchronize()
        g.timing(True)
        g.timing_read("stream_copy", reset=True)
        for _ in range(10):
            g.stream_copy_dev(dbuf, sbuf, nb)
        torch.cuda.synchronize()
        ms, n = g.timing_read("stream_copy", reset=True)
        g.timing(False)
        if n:
            stream_copy = {"GBs": round(2 * nb / (ms / n * 1e-3) / 1e9, 1),
                           "bytes_per_copy": 2 * nb, "copies": n,
                           "kernel": "k_stream_copy (16-B loads/stores, 1 GiB -> 1 GiB)"}
        del sbuf, dbuf
    if ws > 1:
        dist.barrier()  # every rank leaves together (rank 0 ran the copy alone)

    out = None
    if rank == 0:
        ms_per_step = 1000.0 * elapsed / a.steps
        value = job_matches * a.steps / elapsed
        dom_ms, dom_n = kt.get(dom, (0.0, 0))
        dom_avg_us = 1000.0 * dom_ms / max(dom_n, 1)
        roof = None
        if dom_bytes is not None and dom_n > 0:
            ach = dom_bytes / (dom_avg_us * 1e-6) / 1e9
            traffic = build_traffic = None
            if a.traffic_csv:
                traffic = traffic_from_csv(a.traffic_csv.split(","))
                build_traffic = traffic_from_csv(a.traffic_csv.split(","), BUILD_KERNELS)
            else:
                tj = load_traffic(a, {"k": a.k, "points_per_cloud": N})
                if tj is not None:
                    traffic = tj.get("bytes_per_step")
                    build_traffic = tj.get("build_bytes_per_step")
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    # where traffic comes from: this run's PMC CSVs (--traffic-csv),
                    # or the committed json of the round's profiling session
                    "traffic_measured_in_run": bool(a.traffic_csv),
                    "kernel": ("query stage %s<%d> + k_knn_slow<%d>, one launch each per "
                               "step" % (knn_query_kernel(), a.k, a.k)),
                    "avg_us": round(dom_avg_us, 2), "launches": dom_n,
                    "timing": ("HIP events on the context's stream over the timed region"
                               + (f" ({nf} pairs in flight: context 0's launches only, a "
                                  "contended span that also holds the other pairs' "
                                  "interleaved kernels)" if nf > 1 else "")),
                    "bytes_per_launch": dom_bytes,
                    "bytes_model": "24 B/query read + 24 B/target read + 12*k B/query out"}
            tr = load_trace(a, {"k": a.k, "points_per_cloud": N, "knn_mode": knn_mode()})
            if tr is not None and tr.get("trace_us", {}).get("knn_query"):
                # the trace basis (r5): the query stage's kernel
                # durations per launch in the rocprofv3 trace of this command
                q_us = tr["trace_us"]["knn_query"]
                roof["trace"] = {"query_stage_us": q_us, "main_kernel_us": tr.get("main_avg_us"),
                                 "frac": round(dom_bytes / (q_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                                 "source": tr.get("source"), "measured_in_run": False}
            if kt_iso is not None and kt_iso.get(dom, (0, 0))[1] > 0:
                iso_us = 1000.0 * kt_iso[dom][0] / kt_iso[dom][1]
                roof["avg_us_isolated"] = round(iso_us, 2)
                roof["frac_isolated"] = round(dom_bytes / (iso_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
            # the index build is reported separately, outside the
            # headline fraction: its time, the 24 B/target read of the model
            # and its measured traffic
            b_ms, b_n = kt.get("knn_build", (0.0, 0))
            b_iso_n = kt_iso.get("knn_build", (0, 0))[1] if kt_iso is not None else 0
            if b_n or b_iso_n:
                bld = {"kernels": ("k_bbox_partial + k_bin_hist (with the grid) + k_bin_colscan + "
                                   "k_bin_scatter + k_bin_fine (both clouds binned)"
                                   + (" + k_nb_fill (row lists)" if knn_mode() == 2 else "")),
                       # (not timed in the timed region with pairs in flight)
                       "avg_us": round(1000.0 * b_ms / b_n, 2) if b_n else None,
                       "bytes_model": "24 B/target read (SURVEY 8d); the query binning is extra",
                       "algorithmic_bytes": 24 * N, "traffic": build_traffic}
                if kt_iso is not None and kt_iso.get("knn_build", (0, 0))[1] > 0:
                    bld["avg_us_isolated"] = round(
                        1000.0 * kt_iso["knn_build"][0] / kt_iso["knn_build"][1], 2)
                roof["build"] = bld
        elif dom_n > 0:
            roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": None, "traffic": None, "kernel": dom,
                    "avg_us": round(dom_avg_us, 2),
                    "note": "latency/LDS-bound per-row kernel; bytes model in DESIGN.md"}
        if a.workload != "k3" and dom_bytes and dom_n > 0:
            ach = dom_bytes / (dom_avg_us * 1e-6) / 1e9
            tj = load_traffic(a, {"workload": traffic_tag(a), "pairs_per_step": pairs,
                                  "points_per_cloud": N})
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
                    "traffic": tj and tj.get("bytes_per_step"),
                    "kernel": ("rows_match: k_curvature (both clouds) + k_rows_screen (exact "
                               "f64 argmin + runner-up per query) + the tree pass over tied "
                               "rows only"),
                    "avg_us": round(dom_avg_us, 2), "bytes_per_launch": dom_bytes,
                    "bytes_model": ("28 B/point x 2 clouds + 36 B/query + 24 B/target feature "
                                    "(SURVEY 8d)"),
                    "note": ("f64 VALU-bound screen (chunk-box pruned scan); rows with a tie "
                             "add the latency-bound Lomuto tree build (DESIGN.md)")}
        if roof is not None and stream_copy is not None:
            roof["stream_copy"] = stream_copy
            if roof.get("achieved"):
                roof["frac_of_stream_copy"] = round(roof["achieved"] / stream_copy["GBs"], 4)
        path = None
        if path_bytes is not None:
            def path_of(tab, label):
                tot_us = 0.0
                for kname in path_kernels:
                    ms, n = tab.get(kname, (0.0, 0))
                    if n == 0:
                        return None
                    tot_us += 1000.0 * ms / n   # per launch = per pair
                pa = path_bytes / (tot_us * 1e-6) / 1e9
                return {"kernels_us_per_pair": round(tot_us, 2), "bytes_per_pair": path_bytes,
                        "achieved": round(pa, 1), "frac": round(pa / HBM_PEAK_GBS, 4),
                        "timing": label}
            path = path_of(kt, "timed region" + (f", {nf} pairs in flight (contended)"
                                                 if nf > 1 else ""))
            if kt_iso is not None:
                path = dict(path or {}, isolated=path_of(kt_iso, f"{a.iso_steps} steps on one "
                                                        "context after the timed region"))
        cpu = None
        if ws == 1 and not a.no_cpu_baseline and a.workload == "k3":
            cpu = cpu_baseline_k3(src_h, tgt_h, a.k, a.cpu_reps)
        elif rank == 0 and not a.no_cpu_baseline and a.workload in ("k2", "k4") and pairs:
            # one pair of the batch; the reference has no batching (K4 = pairs in turn)
            cpu = cpu_baseline_k2(srcs[0].cpu().numpy(), tgts[0].cpu().numpy(), a.cpu_reps)
        out = {"metric": METRIC, "value": round(value, 1), "unit": "matches/s",
               "n_gpus": ws, "steps": a.steps, "warmup": a.warmup,
               "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": data,
               "config": dict({"workload": workload, "parallelism": f"replicas x{ws}"},
                              **cfg_extra),
               "roofline": roof, "curvature_plus_query": path,
               "kernel_us": {k: (round(1000.0 * v[0] / v[1], 2) if v[1] else None)
                             for k, v in kt.items()},
               "kernel_us_isolated": (None if kt_iso is None else
                                      {k: round(1000.0 * v[0] / max(v[1], 1), 2)
                                       for k, v in kt_iso.items()}),
               "cpu_baseline": cpu}
        if no_gather is not None:
            out["without_gather"] = no_gather
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    g.close()
    for c in (extra if a.workload == "k3" else []):
        c.close()
    if ws > 1:
        dist.destroy_process_group()
    return out


QUERY_KERNELS = ("k_knnw<", "k_knng<", "k_knn_slow<")
# the query pass launched once per step: k_knnw (NAVGPU_KNN_MODE=1) or k_knng
# (2: row neighbourhood lists, r5)
QUERY_MAIN = ("k_knnw<", "k_knng<")
BUILD_KERNELS = ("k_bbox_partial", "k_grid_params", "k_bin_hist", "k_bin_colscan",
                 "k_bin_scatter", "k_bin_fine", "k_nb_fill")
# per-row workloads: the kernels of one step and the kernel launched once per
# step (the per-step divisor)
ROWS_KERNELS = ("k_curvature", "k_rows_screen", "k_rows_match")
K5_KERNELS = ("k_rows_build", "k_rows_query", "k_rows_retree", "k_rows_corr")
TRAFFIC_SETS = {"k3": (QUERY_KERNELS, QUERY_MAIN), "k3_build": (BUILD_KERNELS, QUERY_MAIN),
                "rows": (ROWS_KERNELS, "k_rows_screen"), "k5": (K5_KERNELS, "k_rows_build")}


def traffic_tag(a):
    """profiles/traffic_<tag>.json: the PMC bytes a bench line of this
    workload quotes (k3, k2, k2i, k4, k4i, k5, k5f, k5fl: fast mode with lazy
    row trees, NAVSLAM_HOST_TREES=0)."""
    t = a.workload
    if a.workload in ("k2", "k4") and a.integer_mm:
        t += "i"
    if a.workload == "k5" and a.k5_mode == "fast":
        t += "f"
        if os.environ.get("NAVSLAM_HOST_TREES", "1") == "0":
            t += "l"
    return t


def knn_mode():
    """the K3 query pass the library selects (NAVGPU_KNN_MODE 1 or 2; anything
    else keeps the default 2, as navgpu_create does)"""
    try:
        m = int(os.environ.get("NAVGPU_KNN_MODE", "2"))
    except ValueError:
        return 2
    return m if m in (1, 2) else 2


def knn_query_kernel():
    return "k_knng" if knn_mode() == 2 else "k_knnw"


def load_trace(a, match):
    """profiles/trace_k3.json (scripts/trace_check.py over the round's
    rocprofv3 kernel trace of the default bench command) if its signature
    matches `match`."""
    if a.no_traffic_json:
        return None
    path = os.path.join(ROOT, "profiles", "trace_k3.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        tj = json.load(f)
    if not all(tj.get(k) == v for k, v in match.items()):
        return None
    tj.setdefault("source", os.path.relpath(path, ROOT))
    return tj


def load_traffic(a, match):
    """The traffic json of this workload if its signature matches `match`."""
    if a.no_traffic_json:
        return None
    path = a.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{traffic_tag(a)}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        tj = json.load(f)
    return tj if all(tj.get(k) == v for k, v in match.items()) else None


def pmc_bytes(paths, kernel_subs, anchor=QUERY_MAIN):
    """HBM bytes per step of the kernels whose name contains one of
    `kernel_subs`, from rocprofv3 --pmc counter CSVs (FETCH_SIZE in one pass,
    WRITE_SIZE in another; both in KB). Per step = total / launches of the
    `anchor` kernel (one per step). Returns {"fetch_raw", "write", "bytes"}:
    FETCH_SIZE as counted, WRITE_SIZE, and FETCH_SIZE x 2 (the gfx950
    correction, MI355X_MICROARCH.md HBM section) + WRITE_SIZE."""
    import csv
    fetch, write = 0.0, 0.0
    launches = {}
    for path in paths:
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                c = r.get("Counter_Name")
                if any(x in name for x in ((anchor,) if isinstance(anchor, str) else anchor)):
                    launches.setdefault(c, set()).add(r.get("Dispatch_Id"))
                if not any(k in name for k in kernel_subs):
                    continue
                v = float(r.get("Counter_Value", 0))
                if c == "FETCH_SIZE":
                    fetch += v
                elif c == "WRITE_SIZE":
                    write += v
    nf, nw = len(launches.get("FETCH_SIZE", ())), len(launches.get("WRITE_SIZE", ()))
    if not nf or not nw:
        return None
    return {"fetch_raw": round(fetch / nf * 1024), "write": round(write / nw * 1024),
            "bytes": round((2 * fetch / nf + write / nw) * 1024)}


def traffic_from_csv(paths, kernel_subs=QUERY_KERNELS):
    t = pmc_bytes(paths, kernel_subs)
    return None if t is None else t["bytes"]


if __name__ == "__main__":
    main()
