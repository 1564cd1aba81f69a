#!/usr/bin/env python3
"""Benchmark: IKF iterations/sec, 100k-pt scan vs 10M-pt map (BASELINE.json).

One step = one full scan update (update_iterated_dyn_share_modified) of the
C2 workload in fixed mode: `--iters` (default 4) IKF iterations, each a
device h_share_model pass WITH the 5-NN search + H^T H / H^T h reduction +
the host 24x24 update.  value = IKF iterations/sec of the whole job.

N > 1 (launched by torch.distributed.run): scan points are sharded across
ranks (map replicated), with one RCCL all-reduce of the 8 x 91 fp64
super-chunk sums per iteration (strong scaling: the same 100k scan at every N).

Prints ONE JSON line on rank 0 with `roofline` (dominant kernel = the fused
search pass, timed with HIP events on its own stream over the timed region)
and `cpu_baseline` (the CPU oracle port, 3 OpenMP threads = MP_PROC_NUM).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BYTES_PER_SEARCH_PT = 109   # SURVEY.md §8d compulsory bytes, search pass
BYTES_PER_REUSE_PT = 30     # SURVEY.md §8d compulsory bytes, non-search (reuse) pass
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E peak (MI355X_MICROARCH.md)


L2_PEAK_GBS = 34500.0       # MI355X aggregate L2 read bandwidth (MI355X_MICROARCH.md, L2)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def native_loop():
    """scripts/bench_loop.c -- the C2 step loop as a compiled caller (what
    laserMapping is) -- built next to its source if missing or older than it;
    None when it cannot be built (bench.py then times the Python loop)."""
    import subprocess
    src = os.path.join(ROOT, "scripts", "bench_loop.c")
    so = os.path.join(ROOT, "scripts", "libbench_loop.so")
    try:
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-I", os.path.join(ROOT, "include"), src, "-o",
                            so + ".tmp"], check=True, capture_output=True)
            os.replace(so + ".tmp", so)
        lib = C.CDLL(so)
    except (OSError, subprocess.CalledProcessError) as e:
        log(f"bench.py: no native caller loop ({e}); timing the Python loop")
        return None
    return lib.bench_c2_loop


def l2_demand_bytes(mp: np.ndarray, body: np.ndarray, st0: np.ndarray, cell: float) -> float:
    """Estimated bytes one search launch asks of the L1/L2 (not HBM): per
    query the 2 block-row bounds (8 B), every candidate of its 3x3x3 block
    row (16 B each), the scan point (12 B), the 5 neighbours reloaded by the
    fit (80 B) and the per-point outputs (81 B).  The block is counted on a
    grid of the same cell edge and bounding-box padding as the device map at
    the step's initial pose; refinements and far queries are not counted, so
    this is a lower bound of the kernel's L2-level demand."""
    from agi_lidar_slam_amd import synth
    lo = mp.min(0).astype(np.float64) - 2 * cell
    dims = np.floor((mp.max(0) - lo) / cell).astype(np.int64) + 3
    def cells(p):
        return np.floor((p - lo) / cell).astype(np.int64)
    c = cells(mp.astype(np.float64))
    cnt = np.bincount((c[:, 2] * dims[1] + c[:, 1]) * dims[0] + c[:, 0],
                      minlength=int(np.prod(dims))).reshape(dims[2], dims[1], dims[0])
    R = synth.quat_matrix(st0[3:7])
    q = (body.astype(np.float64) + st0[11:14]) @ R.T + st0[0:3]
    qc = np.clip(cells(q), 1, dims - 2)
    cand = np.zeros(q.shape[0], np.int64)
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                cand += cnt[qc[:, 2] + dz, qc[:, 1] + dy, qc[:, 0] + dx]
    return float(cand.sum() * 16 + q.shape[0] * (8 + 12 + 80 + 81))


def usable_cores() -> tuple[int, str]:
    """Cores this process can actually run on: its affinity set, capped by a
    cgroup CPU quota (the GPU box gives a 1-GPU job a share of a large host:
    nproc and the affinity set show every core, the quota does not)."""
    n = len(os.sched_getaffinity(0))
    why = "affinity set"
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                q = max(1, int(int(quota) // int(period)))
                if q < n:
                    n, why = q, f"cgroup quota {quota}/{period}"
        except (OSError, ValueError):
            pass
    try:  # cgroup v1
        quota = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if quota > 0 and quota // period < n:
            n, why = max(1, quota // period), f"cgroup quota {quota}/{period}"
    except (OSError, ValueError):
        pass
    return n, why


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def frontend_traffic(workload, kernels=None):
    """HBM bytes of one scan through the front-end (every kernel's per-launch
    mean summed; `kernels`: only those) from the committed PMC summary
    (scripts/pmc_frontend.sh: rocprofv3 --pmc cannot run inside this
    process), only when the library was built from the same sources."""
    path = os.path.join(ROOT, "profiles", f"{workload}_traffic.json")
    try:
        tj = json.load(open(path))
        from agi_lidar_slam_amd import build
        if tj.get("workload") == workload and tj.get("source_hash") == build.source_hash():
            if kernels is None:
                return tj.get("hbm_bytes_per_launch")
            pk = tj.get("counters_per_kernel", {})
            if all(k in pk for k in kernels):
                return sum(2 * pk[k]["FETCH_SIZE"] + pk[k]["WRITE_SIZE"] for k in kernels) * 1024
    except (OSError, ValueError, KeyError):
        pass
    return None


# SURVEY.md §8d's compulsory model of a LiDAR front-end scan: per input point
# 22 B in (xyz, intensity, ring, time), 8 B range-image cell, 24 B compacted
# out, ~16 B curvature / flags / labels -> 70 B
FRONTEND_BYTES_PER_PT = 70


def frontend_rooflines(lib, h, args, prefix, points_in, n_ext, nfeat, run_async, workload, feat_kernels):
    """(scan roofline, feature-stage roofline): HIP events in the first and
    last launches of --timing-steps further scans (the whole scan: every
    kernel), then in the feature stage's (k_fe_pick .. k_fe_ring)."""
    from agi_lidar_slam_amd import _lib as L
    prof = getattr(lib, f"{prefix}_profile")
    read = getattr(lib, f"{prefix}_profile_read")
    out = []
    for mode in (L.SLIO_LIO_PROFILE_SCAN, 1):
        prof(h, mode)
        for k in range(max(1, args.timing_steps)):
            L.check(run_async(h), "run_async")
        prof(h, mode | L.SLIO_LIO_PROFILE_KEEP)
        ms, nl = C.c_double(), C.c_int64()
        read(h, C.byref(ms), C.byref(nl))
        prof(h, 0)
        out.append(((ms.value / max(nl.value, 1)) * 1e-3, int(nl.value)))
    (scan_s, scan_n), (feat_s, feat_n) = out
    alg = FRONTEND_BYTES_PER_PT * points_in
    achieved = alg / scan_s / 1e9 if scan_s > 0 else None
    # feature stage (k_fe_pick + k_fe_ring): per extracted point curvature 4 + column 4 +
    # flag 1 + label 4 + the point 16 (surface / corner gathers), and the outputs 16 B each
    falg = 29 * n_ext + 16 * nfeat
    fach = falg / feat_s / 1e9 if feat_s > 0 else None
    scan = {
        "bound": "hbm",
        "kernel": f"the whole scan: every front-end launch ({workload}), first start to last end",
        "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
        "traffic": frontend_traffic(workload),
        "alg_bytes_per_launch": alg,
        "alg_model": f"{FRONTEND_BYTES_PER_PT} B per input point (SURVEY.md 8d)",
        "avg_launch_us": scan_s * 1e6, "launches": scan_n,
        "timing": (f"HIP events in the dispatch packets of the first and last launches of each of "
                   f"{args.timing_steps} further scans"),
    }
    feat = {
        "kernel": "feature stage: k_fe_pick + k_fe_ring (one timed span)",
        "achieved": fach, "frac": (fach / HBM_PEAK_GBS) if fach else None,
        "traffic": frontend_traffic(workload, feat_kernels), "alg_bytes_per_launch": falg,
        "avg_launch_us": feat_s * 1e6, "launches": feat_n,
    }
    return scan, feat


def bench_c3(args, rank, world, dev, dist):
    """C3: LIO-SAM imageProjection + featureExtraction on a
    64 x 2048 Ouster scan (131 072 points).  One step = one scan through the
    whole device front-end with the scan resident in HBM.  N > 1: replicas
    (every rank its own scan stream, no collective): value = scans of all
    ranks / max-over-ranks time."""
    import ctypes as C
    from agi_lidar_slam_amd import _lib as L, build, synth
    from agi_lidar_slam_amd.frontend import LioSamFrontEnd, LioSamParams, imu_deskew_table

    if rank == 0:
        build.build()
    if world > 1:
        dist.barrier()
    L.load()
    S = max(1, args.c3_streams)
    fes, scs = [], []
    for j in range(S):
        # stream j: its own handle, stream and scan (distinct seeds)
        sc_j = synth.make_ouster_scan(seed=20261015 + rank + 7919 * j)
        tb_j = imu_deskew_table(sc_j["imu_stamps"], sc_j["imu_gyro"], sc_j["time_scan_cur"],
                                sc_j["time_scan_end"])
        fe_j = LioSamFrontEnd(LioSamParams(N_SCAN=64, Horizon_SCAN=2048), device=dev)
        fe_j.set_deskew(*tb_j[:4], sc_j["time_scan_cur"], tb_j[4])
        fe_j.upload(sc_j["x"], sc_j["y"], sc_j["z"], sc_j["intensity"], sc_j["ring"], sc_j["time"])
        fes.append(fe_j)
        scs.append((sc_j, tb_j))
    fe = fes[0]
    sc, tb = scs[0]
    lib, h = fe.lib, fe.h
    for _ in range(args.warmup):
        for f in fes:
            f.run()
    counts = L.SlioLioCounts()
    lib.slio_lio_profile(h, 0)
    if world > 1:
        dist.barrier()
    for f in fes:
        L.check(lib.slio_lio_get_counts(f.h, C.byref(counts)), "counts")
    t0 = time.perf_counter()
    for k in range(args.steps):
        for f in fes:  # S scans in flight, one per stream
            rc = lib.slio_lio_run_async(f.h)
            if rc:
                L.check(rc, "slio_lio_run_async")
    for f in fes:
        L.check(lib.slio_lio_get_counts(f.h, C.byref(counts)), "counts")  # waits for each stream
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    L.check(lib.slio_lio_get_counts(h, C.byref(counts)), "counts")
    n_ext, nc, ns = counts.n_extracted, counts.n_corner, counts.n_surface
    # kernel time: HIP events on further scans of stream 0 alone, after the
    # timed region (events cost idle time per launch)
    roof, feat = (None, None)
    if not args.no_kernel_timing:
        roof, feat = frontend_rooflines(lib, h, args, "slio_lio", int(sc["x"].size), n_ext, nc + ns,
                                        lib.slio_lio_run_async, "c3", ["k_fe_pick", "k_fe_ring"])
        if S > 1:
            roof["traffic"] = feat["traffic"] = None
    if world > 1:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    value = args.steps * S * world / el
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        n = max(1, args.cpu_scans_c3)
        t0 = time.perf_counter()
        for _ in range(n):
            info = O.lio_project(sc, 64, 2048, tb)
            O.lio_features(info, 64)
        cel = time.perf_counter() - t0
        cpu = {
            "value": n / cel,
            "unit": "scans/s",
            "cores": 1,
            "kind": "port",
            "sample": (f"{n} scans through the single-threaded C++ restatement of projectPointCloud + "
                       f"cloudExtraction + calculateSmoothness + markOccludedPoints + extractFeatures "
                       f"(+ per-ring VoxelGrid), same 64x2048 Ouster scan; host {cpu_model()}, "
                       f"nproc {os.cpu_count()}"),
        }
    out = {
        "metric": "LIO-SAM imageProjection + featureExtraction scans/sec, 64-ring Ouster 131k-pt scan",
        "value": value,
        "unit": "scans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (points, ranges, curvature) + f64 (deskew interpolation, trig)",
        "streams": S,
        "data": "synthetic (seeded urban scene, OS1-64-like 64 x 2048 sweep with IMU deskew)",
        "config": {
            "workload": ("C3: LIO-SAM ImageProjection::projectPointCloud/cloudExtraction + "
                         "FeatureExtraction::calculateSmoothness/markOccludedPoints/extractFeatures, "
                         "64 x 2048 Ouster scan, deskew on"),
            "points_in": int(sc["x"].size),
            "points_extracted": int(n_ext),
            "corners": int(nc),
            "surface": int(ns),
            "parallelism": ((f"replicas x{world}: one scan stream per GPU, no collective"
                             if world > 1 else "single GPU")
                            + (f"; {S} independent scans in flight per GPU (own handle and stream each)"
                               if S > 1 else "")),
        },
        "roofline": roof,
        "roofline_feature_stage": feat,
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    for f in fes:
        f.close()


def bench_group(args, rank, world, dev, dist):
    """C4 rehearsal on ONE GPU: the drop-in's multi-GPU form
    (slio_create_group / slio_group_ikf_update) with
    --group-ranks ranks sharing this device, so the group takes the in-device
    reduce (k_group_reduce) instead of RCCL over xGMI.  The C2 scan is split
    into the ranks' contiguous shards, the map is shared; one step = one group
    update (--iters passes, fixed flow).  Not the C2 line and not a scaling
    measurement: it times the group path's launches, event waits, reduce and
    filter steps, and (host stamps) where the host spends its time per update."""
    from agi_lidar_slam_amd import _lib as L, build, synth
    build.build()
    lib = L.load()
    n = args.group_ranks
    mp, fr = synth.make_problem(args.map_points, args.scan_points, pattern="avia", cache_dir=args.cache_dir)
    fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
    p = L.SlioParams()
    lib.slio_params_default(C.byref(p))
    p.max_points, p.grid_cell = args.scan_points, args.cell
    hs = (C.c_void_p * n)()
    dv = (C.c_int32 * n)(*([dev] * n))
    L.check(lib.slio_create_group(hs, n, dv, C.byref(p)), "group")
    kind = lib.slio_group_reduce_kind(hs[0])
    x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
    L.check(lib.slio_map_upload(hs[0], L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
    for r in range(1, n):
        L.check(lib.slio_map_share(hs[r], hs[0]), "share")
    bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
    for r in range(n):
        L.check(lib.slio_scan_upload(hs[r], L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
    st0 = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9),
                          [0, 0, -9.81]])
    xs0 = L.SlioState()
    xs0.pos[:] = list(st0[0:3])
    xs0.rot[:] = list(st0[3:7])
    xs0.rli[:] = list(st0[7:11])
    xs0.tli[:] = list(st0[11:14])
    xs0.grav[:] = list(st0[23:26])
    xs = L.SlioState()
    P0 = np.eye(24) * 1e-2
    P = np.empty_like(P0)
    stats = L.SlioIkfStats()

    def step():
        C.memmove(C.addressof(xs), C.addressof(xs0), C.sizeof(xs))
        P[...] = P0
        L.check(lib.slio_group_ikf_update(hs, n, C.byref(xs), L.dptr(P), 0.001, args.iters, 0,
                                          L.SLIO_MODE_FIXED, C.byref(stats)), "group update")

    for _ in range(args.warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    el = time.perf_counter() - t0
    # host stamps of further steps (rank 0's handle)
    hst = np.zeros(8, np.int64)
    lib.slio_debug_host_stamps(hs[0], 1, None)
    rows = []
    for _ in range(max(1, args.timing_steps)):
        step()
        lib.slio_debug_host_stamps(hs[0], -1, L.i64ptr(hst))
        rows.append(hst.copy())
    lib.slio_debug_host_stamps(hs[0], 0, None)
    r = np.array(rows, np.float64) / 1e3
    passes = int(stats.passes)
    # (the fused group path has one launch kind per pass: [4] is all its launches)
    host = {"enqueue_all_us": float(np.median(r[:, 1] - r[:, 0])),
            "rank_pass_launches_us": float(np.median(r[:, 4])),
            "reduce_enqueue_us": float(np.median(r[:, 5])),
            "filter_step_enqueue_us": float(np.median(r[:, 6])),
            "wait_after_enqueue_us": float(np.median(r[:, 2] - r[:, 1])),
            "update_us": float(np.median(r[:, 3] - r[:, 0]))}
    out = {
        "metric": "IKF iterations/sec, C4 group rehearsal on one GPU (not the C2 line)",
        "value": args.steps * passes / el,
        "unit": "IKF iterations/s",
        "n_gpus": 1,
        "group_ranks": n,
        "reduce": {1: "RCCL", 2: "in-device (k_group_reduce)"}.get(kind, str(kind)),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "us_per_pass": el / args.steps / passes * 1e6,
        "host_us_per_update": host,
        "config": {"workload": (f"C4 rehearsal: slio_group_ikf_update, {n} ranks on one device, "
                                f"{args.scan_points}-pt scan split {n} ways vs {args.map_points}-pt map, "
                                f"{args.iters} IKF iterations (fixed flow)"),
                   "map_points": args.map_points, "scan_points": args.scan_points},
        "data": "synthetic (seeded urban scene, Avia-like rosette scan)",
    }
    print(json.dumps(out), flush=True)
    for q in range(n):
        lib.slio_destroy(hs[q])


def bench_lego(args, rank, world, dev, dist):
    """LeGO-LOAM front-end: ImageProjection
    (projectPointCloud, groundRemoval, cloudSegmentation) + the front half of
    FeatureAssociation (adjustDistortion with the IMU ring, calculateSmoothness,
    markOccludedPoints, extractFeatures) on one VLP-16 sweep (16 x 1800, the
    sensor LeGO-LOAM hard-codes, utility.h:53-58), IMU on.  One step = one
    sweep through the whole device pipeline with the sweep resident in HBM.
    N > 1: replicas (no collective)."""
    import ctypes as C
    from agi_lidar_slam_amd import _lib as L, build, synth
    from agi_lidar_slam_amd.lego import LegoFrontEnd, LegoImu, LegoParams

    if rank == 0:
        build.build()
    if world > 1:
        dist.barrier()
    L.load()
    P = LegoParams()
    sw = synth.make_vlp16_sweep(seed=20261015 + rank)
    imu = LegoImu()
    imu.feed(sw["imu"], sw["time_scan_cur"] + 0.15)
    fe = LegoFrontEnd(P, device=dev, max_points=sw["x"].size)
    fe.set_imu(imu, sw["time_scan_cur"])
    fe.upload(sw["x"], sw["y"], sw["z"])
    lib, h = fe.lib, fe.h
    for _ in range(args.warmup):
        fe.run()
    counts = L.SlioLegoCounts()
    lib.slio_lego_profile(h, 0)
    if world > 1:
        dist.barrier()
    L.check(lib.slio_lego_get_counts(h, C.byref(counts)), "counts")
    t0 = time.perf_counter()
    for k in range(args.steps):
        rc = lib.slio_lego_run_async(h)
        if rc:
            L.check(rc, "slio_lego_run_async")
    L.check(lib.slio_lego_get_counts(h, C.byref(counts)), "counts")  # waits for the stream
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    L.check(lib.slio_lego_get_counts(h, C.byref(counts)), "counts")
    nseg = counts.n_segmented
    nfeat = counts.n_sharp + counts.n_less_sharp + counts.n_flat + counts.n_less_flat
    # kernel time (HIP events), further sweeps after the timed region
    roof, feat = (None, None)
    if not args.no_kernel_timing:
        roof, feat = frontend_rooflines(lib, h, args, "slio_lego", int(sw["x"].size), nseg, nfeat,
                                        lib.slio_lego_run_async, "lego", ["k_fe_pick", "k_fe_ring"])
    if world > 1:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    value = args.steps * world / el
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        n = max(1, args.cpu_scans_lego)
        t0 = time.perf_counter()
        for _ in range(n):
            si = O.lego_project(sw["x"], sw["y"], sw["z"], P)
            O.lego_features(si, P, imu, sw["time_scan_cur"])
        cel = time.perf_counter() - t0
        cpu = {
            "value": n / cel,
            "unit": "scans/s",
            "cores": 1,
            "kind": "port",
            "sample": (f"{n} sweeps through the single-threaded C++ restatement of LeGO-LOAM "
                       f"projectPointCloud + groundRemoval + cloudSegmentation + adjustDistortion + "
                       f"calculateSmoothness + markOccludedPoints + extractFeatures (IMU on), same "
                       f"16 x 1800 VLP-16 sweep; host {cpu_model()}, nproc {os.cpu_count()}"),
        }
    out = {
        "metric": "LeGO-LOAM imageProjection + featureAssociation front half scans/sec, VLP-16 16x1800 sweep",
        "value": value,
        "unit": "scans/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (points, ranges, angles, curvature)",
        "data": "synthetic (seeded urban scene, VLP-16 sweep in firing order with a 200 Hz IMU stream)",
        "config": {
            "workload": ("LeGO-LOAM ImageProjection::cloudHandler (projection, ground removal, "
                         "segmentation) + FeatureAssociation adjustDistortion .. extractFeatures, "
                         "16 x 1800 VLP-16 sweep, IMU on"),
            "points_in": int(sw["x"].size),
            "points_segmented": int(nseg),
            "features": {"sharp": int(counts.n_sharp), "less_sharp": int(counts.n_less_sharp),
                         "flat": int(counts.n_flat), "less_flat": int(counts.n_less_flat)},
            "parallelism": (f"replicas x{world}: one sweep stream per GPU, no collective"
                            if world > 1 else "single GPU"),
        },
        "roofline": roof,
        "roofline_feature_stage": feat,
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    fe.close()


def bench_c5(args, rank, world, dev, dist):
    """C5 (BASELINE config 5): batched replay -- `--replicas`
    DIFFERENT 100k-point scans in flight at once per GPU against one shared
    50M-point map (agi_lidar_slam_amd.replay: one handle, stream and host
    thread per scan, slio_map_share).  Replicas only: every rank replays its
    own scans against its own map replica, no collective (weak scaling: 4
    per GPU, 32 on 8 GPUs).  One step = one full update (4 IKF iterations) of
    every replica; value = IKF iterations of all replicas of all ranks / the
    max-over-ranks time.  Every replica's x and P are checked bitwise against
    its own update run alone before the timed region."""
    from agi_lidar_slam_amd import build, replay
    import torch

    if rank == 0:
        build.build()
    if world > 1:
        dist.barrier()
    t0 = time.time()
    mp, frames = replay.replay_frames(args.map_points, args.scan_points, args.replicas,
                                      cache_dir=args.cache_dir, first=rank * args.replicas)
    log(f"[rank {rank}] map {mp.shape[0]} + {len(frames)} scans in {time.time() - t0:.1f}s")
    rp = replay.Replay(mp, frames, device=dev, iters=args.iters, cell=args.cell)
    cell_m = rp.cell()
    rp.verify()
    single = rp.solo_rate(max(10, args.steps // 4), args.warmup) if rank == 0 else None

    def before():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def after(el):
        torch.cuda.synchronize()
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    el = rp.run(args.steps, args.warmup, before, after)
    same = rp.identical()
    if world > 1:
        t = torch.tensor([1 if same else 0], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        same = bool(t.item())
    rp.close()
    total = world * args.replicas * args.steps * args.iters / el
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        t0 = time.time()
        T = O.Tree(mp)
        log(f"[cpu] oracle kd-tree built in {time.time() - t0:.1f}s")
        n = max(1, args.cpu_scans_c5)
        t0 = time.perf_counter()
        for k in range(n):
            fr = frames[k % len(frames)]
            st0 = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth_t_li(), np.zeros(9),
                                  [0, 0, -9.81]])
            O.ikf_update(T, fr.body, st0, np.eye(24) * 1e-2, maximum_iter=args.iters, mode=1,
                         reference_gain=1, threads=args.cpu_threads)
        cel = time.perf_counter() - t0
        cpu = {"value": n * args.iters / cel, "unit": "IKF iterations/s", "cores": args.cpu_threads,
               "kind": "port",
               "sample": (f"{n} scan updates x {args.iters} IKF iterations of the replay's scans, one at a "
                          f"time, vs the {args.map_points}-pt map, {args.cpu_threads} OpenMP threads; host "
                          f"{cpu_model()}")}
    out = {
        "metric": "IKF iterations/sec, batched replay of concurrent 100k-pt scans vs a shared 50M-pt map",
        "value": total,
        "unit": "IKF iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (kNN, plane) + f64 (Jacobian, reduction, 24x24 update)",
        "data": "synthetic (seeded urban scene, distinct Avia-like rosette scans)",
        "config": {
            "workload": (f"C5: {args.replicas} concurrent distinct {args.scan_points}-pt scans per GPU vs a shared "
                         f"{args.map_points}-pt map, {args.iters} IKF iterations per update, kNN every "
                         "iteration"),
            "map_points": args.map_points,
            "scan_points": args.scan_points,
            "replicas_per_gpu": args.replicas,
            "grid_cell_m": cell_m,
            "parallelism": (f"replicas: {args.replicas} per GPU x {world} GPUs, map replica per GPU, "
                            "no collective"),
            "results_identical_to_solo_runs": same,
            "single_replica_value": single,
        },
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if not same:
        raise SystemExit("C5: a concurrent replica's result differs from its solo run")


def bench_s2m(args, rank, world, dev, dist):
    """LIO-SAM mapOptimization::scan2MapOptimization (mapOptmization.cpp:
    1706-1740) on the device: per LM iteration
    cornerOptimization + surfOptimization (pointAssociateToMap, exact 5-NN in
    the corner / surf local maps, line / plane fits, :1303-1515), the
    LMOptimization normal equations on the device (:1552-1626) and the 6 x 6
    step on the host (slio_s2m_lm_step).  One step = one scan2MapOptimization
    call from the same perturbed prior to convergence (<= 30 iterations, the
    reference's loop); value = LM iterations/s (and scans/s).  N > 1:
    replicas (no collective)."""
    from agi_lidar_slam_amd import _lib as L, build, synth
    from agi_lidar_slam_amd.lio_sam import ScanToMap

    if rank == 0:
        build.build()
    if world > 1:
        dist.barrier()
    L.load()
    pr = synth.make_s2m_problem()
    s = ScanToMap(max_points=max(pr["surf_scan"].shape[0], pr["corner_scan"].shape[0]), device=dev)
    s.set_maps(pr["corner_map"], pr["surf_map"])
    s.set_scan(pr["corner_scan"], pr["surf_scan"])
    tf0 = pr["tf"] + np.array([0.005, -0.004, 0.01, 0.15, -0.1, 0.05], np.float32)
    lib = s.lib
    for _ in range(args.warmup):
        s.scan2MapOptimization(tf0)
    iters = s.iterations
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tf = s.scan2MapOptimization(tf0)
    el = time.perf_counter() - t0
    assert s.iterations == iters
    # the dominant kernel's time (HIP events on the kNN passes, SLIO_KERNEL_SEARCH) and
    # the whole iteration's device time, over further steps after the timed region
    ms, nl = C.c_double(), C.c_int64()
    search_bit = 1 << (L.SLIO_KERNEL_SEARCH + 1)
    per_kernel = {}
    if not args.no_kernel_timing:
        for h in (s.hc, s.hs):
            lib.slio_profile(h, search_bit)
        for _ in range(max(1, args.timing_steps // 4)):
            s.scan2MapOptimization(tf0)
        for name, h in (("corner", s.hc), ("surf", s.hs)):
            lib.slio_profile(h, search_bit | L.SLIO_PROFILE_KEEP)
            lib.slio_profile_read(h, L.SLIO_KERNEL_SEARCH, C.byref(ms), C.byref(nl))
            per_kernel[name] = (ms.value, nl.value)
            lib.slio_profile(h, 0)
    if world > 1:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    nc, ns = pr["corner_scan"].shape[0], pr["surf_scan"].shape[0]
    value = args.steps * iters * world / el
    # kNN pass (slio_s2m_coeffs' search launch, kNN-only): per query point the
    # point (12 B), its 5 neighbours (80 B with the map index), the neighbour
    # positions, ids and distances written (60 B)
    alg = {"corner": 152 * nc, "surf": 152 * ns}
    roof = None
    if per_kernel and per_kernel["surf"][1] > 0:
        avg_s = per_kernel["surf"][0] / per_kernel["surf"][1] * 1e-3
        achieved = alg["surf"] / avg_s / 1e9
        roof = {"bound": "hbm", "kernel": "k_search_pass (kNN-only: the surf cloud's 5-NN per LM iteration)",
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": None, "alg_bytes_per_launch": alg["surf"], "avg_launch_us": avg_s * 1e6,
                "launches": int(per_kernel["surf"][1]),
                "corner_launch_us": (per_kernel["corner"][0] / max(per_kernel["corner"][1], 1)) * 1e3,
                "timing": "HIP events in the dispatch packet of the kNN launches of further calls"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        Tc, Ts = O.Tree(pr["corner_map"]), O.Tree(pr["surf_map"])
        n = max(1, args.cpu_s2m_iters)
        tfc = tf0.copy()
        t0 = time.perf_counter()
        for _ in range(n):
            clouds = []
            for kind, T, body, mp in ((0, Tc, pr["corner_scan"], pr["corner_map"]),
                                      (1, Ts, pr["surf_scan"], pr["surf_map"])):
                wpt = O.s2m_transform(tfc, body)
                idx, sqd = T.knn(wpt, 5, threads=1)
                cf, sl = O.s2m_coeffs(kind, wpt, mp, idx, sqd)
                clouds.append((body, cf, sl))
            O.s2m_normal_equations(tfc, clouds)
        cel = time.perf_counter() - t0
        cpu = {"value": n / cel, "unit": "LM iterations/s", "cores": 1, "kind": "port",
               "sample": (f"{n} LM iterations (pointAssociateToMap + kd-tree 5-NN + corner / surf "
                          f"coefficients + normal equations, {nc} corner + {ns} surf points) of the "
                          f"single-threaded C++ restatement; host {cpu_model()}")}
    out = {
        "metric": "LIO-SAM scan2MapOptimization LM iterations/sec",
        "value": value,
        "unit": "LM iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "scans_per_s": args.steps * world / el,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (kNN, fits, coefficients) + f64 (normal-equation sums)",
        "data": "synthetic (seeded urban scene: surf map sampled from its surfaces, corner map along its "
                "vertical edges; Avia-like surf scan)",
        "config": {
            "workload": (f"LIO-SAM scan2MapOptimization: {nc} corner + {ns} surf points vs a "
                         f"{pr['corner_map'].shape[0]}-pt corner map and a {pr['surf_map'].shape[0]}-pt "
                         f"surf map, {iters} LM iterations to convergence"),
            "lm_iterations_per_step": iters,
            "degenerate": int(s.isDegenerate.value),
            "final_error_m": float(np.abs(tf[3:] - pr["tf"][3:]).max()),
            "parallelism": (f"replicas x{world}, no collective" if world > 1 else "single GPU"),
        },
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    s.close()


def synth_t_li():
    from agi_lidar_slam_amd import synth
    return synth.AVIA_T_LI


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def resolve_gpus(args, argv=None):
    """--gpus N against the launch (before anything touches a GPU):

    * under torch.distributed.run (WORLD_SIZE set): N must equal WORLD_SIZE;
      with the nccl backend every local rank needs a device of its own;
    * a plain `bench.py --gpus N`, N > 1: the N ranks are started here, one
      process per GPU, by torch.distributed.run in a child process (the
      driver's own launch; this process never initialises a GPU, then exits
      with the child's status);
    * N must not exceed the visible devices (torch.cuda.device_count() does
      not initialise the GPU on this image): a run that cannot place its ranks
      exits non-zero instead of printing a line measured on fewer GPUs.

    Returns None to go on in this process, else the exit status."""
    import subprocess
    if args.gpus < 1:
        log(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
        return 2
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        world = int(env_world)
        if world != args.gpus:
            log(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world} (one rank per GPU)")
            return 2
        if world > 1 and args.dist_backend == "nccl":
            import torch
            local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
            ndev = torch.cuda.device_count()
            if ndev < local_world:
                log(f"bench.py: {local_world} ranks on this node need {local_world} GPUs, {ndev} visible")
                return 2
        return None
    if args.gpus == 1:
        return None
    import torch
    ndev = torch.cuda.device_count()
    if ndev < args.gpus and args.dist_backend == "nccl":
        log(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, {ndev} visible")
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)]
    cmd += list(sys.argv[1:] if argv is None else argv)
    log(f"bench.py: --gpus {args.gpus}: one rank per GPU via {' '.join(cmd[1:6])} ...")
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--iters", type=int, default=4,
                    help="maximum_iter of each update (C2: 4; the Avia launch file's is 3)")
    ap.add_argument("--mode", choices=["fixed", "reference"], default="fixed",
                    help="fixed: exactly --iters passes, kNN every pass (the C2 throughput line); "
                         "reference: the esekfom.hpp:292-345 control flow (passes i = -1 .. iters-1, "
                         "a kNN only after converged passes, reuse passes between), what the drop-in "
                         "runs (mapping_avia.launch:11: --iters 3)")
    ap.add_argument("--map-points", type=int, default=None,
                    help="default: 10M (c2), 50M (c5)")
    ap.add_argument("--scan-points", type=int, default=100_000)
    ap.add_argument("--cell", type=float, default=0.0,
                    help="map grid cell edge (speed only; results are exact at any edge); 0: the "
                         "library's auto edge, 1.0 m at C2 (the sweep's best, profiles/r02_cell_sweep.log)")
    ap.add_argument("--scan-order", choices=["voxel", "capture"], default="voxel",
                    help="voxel: pcl::VoxelGrid output order, as feats_down_body reaches "
                         "h_share_model in the reference; capture: rosette firing order")
    ap.add_argument("--cpu-scans", type=int, default=12)
    ap.add_argument("--cpu-threads", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no HIP events on the search kernel (roofline fields null)")
    ap.add_argument("--timing-steps", type=int, default=40,
                    help="c2: steps after the timed region whose search launches carry HIP events "
                         "(roofline.avg_launch_us)")
    ap.add_argument("--caller", choices=["native", "python"], default="native",
                    help="c2: the timed step loop in C (scripts/bench_loop.c, the laserMapping-style "
                         "caller) or in Python (ctypes per step)")
    ap.add_argument("--no-python-reference", action="store_true",
                    help="c2: skip timing the Python loop beside the native one")
    ap.add_argument("--host-loop", action="store_true",
                    help="run the 24x24 step on the host after every pass (slio_ikf_update)")
    ap.add_argument("--cache-dir", default=os.environ.get("SLIO_CACHE", "/tmp/slio_cache"))
    ap.add_argument("--group-ranks", type=int, default=8,
                    help="group: ranks of the one-GPU C4 rehearsal (must divide 8)")
    ap.add_argument("--workload", choices=["c2", "c3", "c5", "lego", "group", "s2m"], default="c2",
                    help="c2: IKF iterations/s, 100k Avia scan vs 10M map (BASELINE.json metric); "
                         "c3: LIO-SAM front-end scans/s on a 64 x 2048 Ouster scan; "
                         "c5: batched replay, --replicas concurrent distinct 100k scans per GPU vs a "
                         "shared 50M map (BASELINE config 5: 32 scans on 8 GPUs = 4 per GPU); "
                         "lego: LeGO-LOAM front-end scans/s on a VLP-16 16 x 1800 sweep, IMU on; "
                         "group: the C4 group path (slio_group_ikf_update) rehearsed with --group-ranks "
                         "ranks on one GPU; s2m: LIO-SAM scan2MapOptimization LM iterations/s")
    ap.add_argument("--replicas", type=int, default=4, help="c5: concurrent scans per GPU")
    ap.add_argument("--cpu-scans-c5", type=int, default=4)
    ap.add_argument("--reduce-hook", action="store_true",
                    help="N > 1: all-reduce through a torch.distributed hook (slio_allreduce_fn) "
                         "instead of the library's own RCCL communicator (slio_comm_init); implied by "
                         "--dist-backend gloo (RCCL refuses two ranks on one device)")
    ap.add_argument("--cpu-scans-c3", type=int, default=300)
    ap.add_argument("--cpu-s2m-iters", type=int, default=40)
    ap.add_argument("--cpu-scans-lego", type=int, default=300)
    ap.add_argument("--c3-streams", type=int, default=1,
                    help="c3: independent scans in flight per GPU, each on its own handle and stream "
                         "(1: one scan stream, the latency-bound rate)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse the multi-rank path with several ranks on one GPU)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "search_traffic.json"))
    args = ap.parse_args()

    rc = resolve_gpus(args)
    if rc is not None:
        raise SystemExit(rc)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    # one rank per GPU; the modulo only matters for a gloo rehearsal with more
    # ranks than devices (device_count() does not initialise the GPU here)
    dev = local_rank % max(1, torch.cuda.device_count()) if world > 1 else 0
    if args.map_points is None:
        args.map_points = 50_000_000 if args.workload == "c5" else 10_000_000
    if world > 1:
        torch.cuda.set_device(dev)
        dist.init_process_group(args.dist_backend if args.workload == "c2" else "gloo")
    if args.workload in ("c3", "c5", "lego", "group", "s2m"):
        {"c3": bench_c3, "c5": bench_c5, "lego": bench_lego, "group": bench_group, "s2m": bench_s2m}[args.workload](
            args, rank, world, dev, dist)
        if world > 1:
            dist.destroy_process_group()
        return

    from agi_lidar_slam_amd import _lib as L, build, synth

    if rank == 0:
        build.build()
    if world > 1:
        dist.barrier()
    lib = L.load()

    t0 = time.time()
    mp, fr = synth.make_problem(args.map_points, args.scan_points, pattern="avia",
                                cache_dir=args.cache_dir)
    if args.scan_order == "voxel":
        fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
    log(f"[rank {rank}] synthetic problem {mp.shape[0]} map / {fr.body.shape[0]} scan "
        f"in {time.time() - t0:.1f}s")

    p = L.SlioParams()
    lib.slio_params_default(C.byref(p))
    p.device, p.max_points, p.rank, p.nranks = dev, args.scan_points, rank, world
    p.grid_cell = args.cell
    h = C.c_void_p()
    L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
    x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
    t0 = time.time()
    L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
    log(f"[rank {rank}] map index built in {time.time() - t0:.2f}s")
    cell_m = C.c_float()
    L.check(lib.slio_map_info(h, None, C.byref(cell_m), None), "map_info")
    cell_m = float(cell_m.value)  # the edge the library chose
    bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
    L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
    b, e = C.c_int64(), C.c_int64()
    lib.slio_shard_range(h, C.byref(b), C.byref(e))
    shard_pts = e.value - b.value

    reduce_cb = L.ALLREDUCE_FN()
    keep = []
    comm = "none"
    if world > 1 and not args.reduce_hook and args.dist_backend == "nccl":
        # the library's own communicator: rank 0's RCCL id to every rank,
        # then each pass's all-reduce is enqueued inside slio_ikf_update_device
        uid = (C.c_uint8 * L.SLIO_COMM_ID_BYTES)()
        if rank == 0:
            L.check(lib.slio_comm_unique_id(uid), "comm id")
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (C.c_uint8 * L.SLIO_COMM_ID_BYTES).from_buffer_copy(obj[0])
        L.check(lib.slio_comm_init(h, uid), "comm init")
        comm = "library RCCL communicator (slio_comm_init), one ncclAllReduce per iteration"
    elif world > 1:
        # the library and the collective must share one stream: a stream of
        # our own made current (torch's default stream is handle 0, which
        # slio_set_stream reads as "the handle's own stream")
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)
        lib.slio_set_stream(h, C.c_void_p(stream.cuda_stream))
        sup = torch.zeros(8 * 91, dtype=torch.float64, device=f"cuda:{dev}")
        lib.slio_set_super_buffer(h, C.c_void_p(sup.data_ptr()))

        def _allreduce(ctx, buf, count, strm):
            dist.all_reduce(sup, op=dist.ReduceOp.SUM)
            return 0

        reduce_cb = L.ALLREDUCE_FN(_allreduce)
        keep.append(reduce_cb)
        comm = (f"torch.distributed {args.dist_backend} all_reduce through a slio_allreduce_fn hook"
                + (" (RCCL)" if args.dist_backend == "nccl" else ""))

    st0 = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9),
                          [0, 0, -9.81]])
    P0 = np.eye(24) * 1e-2
    stats = L.SlioIkfStats()

    xs0 = L.SlioState()
    xs0.pos[:] = list(st0[0:3])
    xs0.rot[:] = list(st0[3:7])
    xs0.rli[:] = list(st0[7:11])
    xs0.tli[:] = list(st0[11:14])
    xs0.grav[:] = list(st0[23:26])
    xs = L.SlioState()
    P = np.empty_like(P0)
    P_ptr, xs_ref, st_ref = L.dptr(P), C.byref(xs), C.byref(stats)
    fn = lib.slio_ikf_update if args.host_loop else lib.slio_ikf_update_device
    mode = L.SLIO_MODE_REFERENCE if args.mode == "reference" else L.SLIO_MODE_FIXED
    P0c = np.ascontiguousarray(P0)
    xs_a, xs0_a, xs_n = C.addressof(xs), C.addressof(xs0), C.sizeof(xs)
    P_a, P0_a, P_n = P.ctypes.data, P0c.ctypes.data, P.nbytes
    R_c, it_c, ext_c, mode_c = C.c_double(0.001), C.c_int(args.iters), C.c_int(0), C.c_int(mode)

    def step():
        # every step restarts from the same prior (same work per step): x and
        # P copied back by memmove, the call's scalars prebuilt
        C.memmove(xs_a, xs0_a, xs_n)
        C.memmove(P_a, P0_a, P_n)
        rc = fn(h, xs_ref, P_ptr, R_c, it_c, ext_c, mode_c, reduce_cb, None, st_ref)
        if rc:
            L.check(rc, "ikf")
        return xs

    # the timed loop: the compiled caller (scripts/bench_loop.c) unless
    # --caller python; each step copies the prior in and runs one update
    loop = native_loop() if args.caller == "native" else None
    if loop is not None:
        loop.restype = C.c_int
        loop.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(L.SlioState), C.POINTER(C.c_double), C.c_double,
                         C.c_int, C.c_int, C.c_int, L.ALLREDUCE_FN, C.c_void_p, C.c_int64,
                         C.POINTER(L.SlioState), C.POINTER(C.c_double), C.POINTER(L.SlioIkfStats)]
        fn_addr = C.cast(fn, C.c_void_p)
        P0_ptr = L.dptr(P0c)

    def run(k):
        if loop is None:
            for _ in range(k):
                step()
            return
        rc = loop(fn_addr, h, C.byref(xs0), P0_ptr, R_c, it_c, ext_c, mode_c, reduce_cb, None, k, xs_ref, P_ptr,
                  st_ref)
        if rc:
            L.check(rc, "ikf")

    # the roofline's per-launch kernel time first: HIP events in the dispatch
    # packets of every search launch of --timing-steps steps of the same work
    # (events cost ~5 us of idle per launch, so they stay out of the steps
    # `value` is measured on).  Run BEFORE the warmup, they also bring the GPU
    # out of idle: the driver's short setting (--steps 20 --warmup 5) read
    # ~3 % low from clock ramp-up alone when they ran after the timed region.
    search_bit = 1 << (L.SLIO_KERNEL_SEARCH + 1)
    ms = C.c_double()
    nl = C.c_int64()
    lib.slio_profile(h, 0)  # reset totals
    if not args.no_kernel_timing:
        # (a fresh map index gets its block rows after 8 unchanged search
        # passes, kBlkAfterPasses: those updates stay out of the timing)
        for _ in range(3):
            step()
        lib.slio_profile(h, search_bit)
        for k in range(max(1, args.timing_steps)):
            step()
        lib.slio_profile(h, search_bit | L.SLIO_PROFILE_KEEP)
        lib.slio_profile_read(h, L.SLIO_KERNEL_SEARCH, C.byref(ms), C.byref(nl))
    lib.slio_profile(h, 0)
    run(args.warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    # the same steps from the Python loop, for reference (not `value`)
    py_el = None
    if loop is not None and not args.no_python_reference:
        npy = min(args.steps, 100)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(npy):
            step()
        torch.cuda.synchronize()
        py_el = (time.perf_counter() - t1) / npy
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # passes per update: --iters in fixed mode; in the reference flow what the
    # control flow ran (the same every step: same inputs)
    passes, searches = int(stats.passes), int(stats.searches)
    iters_total = args.steps * passes
    value = iters_total / el
    avg_kernel_s = (ms.value / max(nl.value, 1)) * 1e-3
    # algorithmic bytes per launch: a pass is a search (109 B/pt) or, in the
    # reference flow, a reuse (30 B/pt); the persistent update runs every pass
    # of an update in one launch, the per-pass path one pass per launch
    persistent = (world == 1 and not args.host_loop and hasattr(lib, "slio_debug_update_path")
                  and lib.slio_debug_update_path(h) == 1)
    alg_bytes = (searches * BYTES_PER_SEARCH_PT + (passes - searches) * BYTES_PER_REUSE_PT) * shard_pts
    if not persistent:
        alg_bytes /= passes
    achieved = alg_bytes / avg_kernel_s / 1e9 if avg_kernel_s > 0 else None
    # x and P of the last update (every rank holds the same bits): lets a
    # multi-rank run be compared with a single-rank one
    import hashlib
    digest = hashlib.sha256(C.string_at(C.addressof(xs), C.sizeof(xs)) + P.tobytes()).hexdigest()[:16]
    # every iteration's 5 nearest are exact: searched in full, or certified from
    # the update's earlier search (kNN certificates).  Per pass from updates of
    # 1 .. maxit passes from the same prior (fixed flow: the same first passes),
    # after the timed region: the counters cost two atomics per workgroup
    knn = {"label": "exact 5-NN every iteration (searched or certified)"}
    if args.mode == "fixed" and not args.host_loop and world == 1 and hasattr(lib, "slio_debug_knn_cert"):
        cc = (C.c_uint32 * 2)()
        L.check(lib.slio_debug_knn_cert(h, cc), "knn_cert")
        cert, srch = [], []
        for k in range(1, args.iters + 1):
            it_c.value = k
            a0, a1 = int(cc[0]), int(cc[1])
            step()
            L.check(lib.slio_debug_knn_cert(h, cc), "knn_cert")
            cert.append((int(cc[0]) - a0) % (1 << 32))
            srch.append((int(cc[1]) - a1) % (1 << 32))
        it_c.value = args.iters
        cert_pass = [cert[0]] + [cert[k] - cert[k - 1] for k in range(1, len(cert))]
        srch_pass = [srch[0]] + [srch[k] - srch[k - 1] for k in range(1, len(srch))]
        srch_pass[0] = shard_pts  # pass 0 searches every query (no certificate to use)
        knn["certified_per_pass"] = cert_pass
        knn["searched_in_full_per_pass"] = srch_pass
    # HBM bytes per launch from the committed PMC summary (rocprofv3 --pmc
    # cannot run inside this process): only for the same workload, one rank
    # holding the whole scan, and the library built from the same sources
    traffic = None
    if (os.path.exists(args.traffic_json) and world == 1 and shard_pts == args.scan_points
            and args.mode == "fixed"):
        try:
            tj = json.load(open(args.traffic_json))
            if (tj.get("scan_points") == args.scan_points and tj.get("map_points") == args.map_points
                    and tj.get("source_hash") == build.source_hash()):
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    l2 = None
    if rank == 0 and avg_kernel_s > 0 and args.mode == "fixed":
        dem = l2_demand_bytes(mp, fr.body[b.value:e.value], st0, cell_m) * (passes if persistent else 1)
        l2 = {"demand_bytes_per_launch": dem, "achieved": dem / avg_kernel_s / 1e9,
              "peak": L2_PEAK_GBS, "unit": "GB/s", "frac": dem / avg_kernel_s / 1e9 / L2_PEAK_GBS,
              "note": "L2-level roofline of the same launches: block-row candidates + "
                      "neighbour reloads + outputs per query (bench.l2_demand_bytes, a lower "
                      "bound: refinements not counted) / avg launch time, vs the L2 bandwidth"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        t0 = time.time()
        T = O.Tree(mp)
        log(f"[cpu] oracle kd-tree built in {time.time() - t0:.1f}s")
        t0 = time.perf_counter()
        for _ in range(args.cpu_scans):
            _, _, cst, *_ = O.ikf_update(T, fr.body, st0, P0, maximum_iter=args.iters, mode=mode,
                                         reference_gain=1, threads=args.cpu_threads)
        cel = time.perf_counter() - t0
        cpu_passes = int(cst[0])
        # the same sample on every core this process may use (the reference's
        # MP_PROC_NUM is 3; SURVEY.md 8(d) asks for both)
        all_cores, cores_why = usable_cores()
        t0 = time.perf_counter()
        for _ in range(args.cpu_scans):
            O.ikf_update(T, fr.body, st0, P0, maximum_iter=args.iters, mode=mode,
                         reference_gain=1, threads=all_cores)
        cel_all = time.perf_counter() - t0
        cpu = {
            "value": args.cpu_scans * cpu_passes / cel,
            "unit": "IKF iterations/s",
            "all_cores": {"value": args.cpu_scans * cpu_passes / cel_all, "cores": all_cores},
            "cores": args.cpu_threads,
            "kind": "port",
            "sample": (f"{args.cpu_scans} scan updates x {cpu_passes} IKF iterations ("
                       + ("kNN every iteration" if args.mode == "fixed" else
                          f"reference control flow, maximum_iter {args.iters}, {int(cst[1])} kNN passes")
                       + ", 24 x m gain formed as esekfom.hpp:314), "
                       f"{args.scan_points}-pt scan vs {args.map_points}-pt map, "
                       f"{args.cpu_threads} OpenMP threads (MP_PROC_NUM), and all_cores = every "
                       f"core this process may use ({cores_why}); host {cpu_model()}, "
                       f"nproc {os.cpu_count()}"),
        }

    flow = (f"{args.iters} IKF iterations per step with the 5-NN search every iteration"
            if args.mode == "fixed" else
            f"reference control flow (esekfom.hpp:292-345, maximum_iter {args.iters}): {passes} IKF "
            f"iterations per step, {searches} with the 5-NN search")
    out = {
        "metric": "IKF iterations/sec, 100k-pt scan vs 10M-pt map",
        "value": value,
        "unit": "IKF iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32 (kNN, plane) + f64 (Jacobian, reduction, 24x24 update)",
        "data": "synthetic (seeded urban scene, Avia-like rosette scan)",
        "config": {
            "workload": ("C2: S-FAST_LIO update_iterated_dyn_share_modified, "
                         f"{args.scan_points}-pt Avia scan vs {args.map_points}-pt map, " + flow),
            "map_points": args.map_points,
            "scan_points": args.scan_points,
            "iterations_per_step": passes,
            "control_flow": args.mode,
            "maximum_iter": args.iters,
            "searches_per_step": searches,
            "ikf_loop": "host" if args.host_loop else "device-resident",
            "grid_cell_m": cell_m,
            "parallelism": (f"scan points sharded x{world}, map replicated, one all-reduce of 8x91 fp64 "
                            f"per iteration: {comm}" if world > 1 else "single GPU"),
            "effective_points": int(stats.last_m),
            "caller": ("native: scripts/bench_loop.c calls slio_ikf_update_device once per step, as "
                       "laserMapping's C++ loop does" if loop is not None else "Python ctypes loop"),
            "python_loop_value": (passes / py_el) if py_el else None,
            "knn": knn,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": (("k_update_persist (one launch per update: every pass, each summed and followed "
                        "by its filter step inside the launch"
                        if persistent else
                        "k_search_pass (fused: each launch also sums the pass and runs its filter step")
                       + ("" if args.mode == "fixed" else "; search or reuse pass as the update decides")
                       + ")"),
            "launch_covers": f"{passes} passes" if persistent else "1 pass",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": traffic,
            "alg_bytes_per_launch": alg_bytes,
            "avg_launch_us": avg_kernel_s * 1e6,
            "launches": int(nl.value),
            "timing": (f"HIP events in the dispatch packet of every search launch of {args.timing_steps} "
                       "steps of the same work before the warmup and the timed region"),
        },
        "roofline_l2": l2,
        "cpu_baseline": cpu,
        "result_digest": digest,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    lib.slio_destroy(h)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
