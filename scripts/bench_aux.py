#!/usr/bin/env python3
"""Timings of the rows around the hot path on one GPU.

  mapping   live laserMapping per scan on the C2-size map: lasermap_fov_segment +
            Delete_Point_Boxes, the 4-iteration device IKF update, map_incremental,
            and the device index rebuild the next search needs (forced here)
  preproc   UndistortPcl back-propagation + downSizeFilterSurf of a raw scan
  s2m       one LIO-SAM scan-to-map iteration (corner + surf coefficients, normal
            equations, LM step)
One JSON line per measurement (host wall clock around synchronous calls)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def t_ms(f, reps=1):
    t0 = time.perf_counter()
    for _ in range(reps):
        r = f()
    return (time.perf_counter() - t0) * 1e3 / reps, r


def mapping(n_map, n_scan, frames_n=6):
    from agi_lidar_slam_amd import _lib as L, synth
    from agi_lidar_slam_amd.esekf import StateIkfom
    from agi_lidar_slam_amd.mapping import LaserMapping
    seed = 20261015
    mp, _ = synth.make_problem(n_map, n_scan, cache_dir="/tmp/slio_cache")
    frames = synth.make_trajectory(seed, n_map, frames_n, n_scan, step=0.5)
    lm = LaserMapping(max_points=n_scan, cube_len=1000.0)
    lm.ikdtree.set_downsample_param(0.5)
    lm.ikdtree.Build(mp)
    lm.built = True
    lm.first_lidar_time = 0.0
    x = StateIkfom(pos=frames[0].gt_pos.copy(), rot=frames[0].gt_rot.copy(), offset_T_L_I=synth.AVIA_T_LI.copy())
    lm.kf.change_x(x)
    lib = L.load()
    rows = []
    steps, search = [], []
    for k, fr in enumerate(frames):
        x = lm.kf.get_x()
        if k:
            x.pos = x.pos + (fr.gt_pos - frames[k - 1].gt_pos)
            if os.environ.get("MAPPING_PRIOR") == "gtrot":
                # diagnostic: the ground-truth rotation as well (the default
                # prior carries the previous scan's rotation)
                x.rot = fr.gt_rot.copy()
        lm.kf.change_x(x)
        lm.kf.change_P(np.eye(24) * 1e-2)
        body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
        # HIP events on this scan's search launches (diagnostic: ~5 us per launch)
        lib.slio_profile(lm.kf.h, 1 << (L.SLIO_KERNEL_SEARCH + 1))
        t0 = time.perf_counter()
        lm.process(body, lidar_beg_time=0.1 * (k + 1))
        t_total = (time.perf_counter() - t0) * 1e3
        ms, nl = C.c_double(), C.c_int64()
        lib.slio_profile_read(lm.kf.h, L.SLIO_KERNEL_SEARCH, C.byref(ms), C.byref(nl))
        lib.slio_profile(lm.kf.h, 0)
        nfar = C.c_int64()
        lib.slio_far_queries(lm.kf.h, C.byref(nfar))
        n = C.c_int64()
        t_rebuild, _ = t_ms(lambda: lib.slio_map_info(lm.ikdtree.h, None, None, C.byref(n)))
        rows.append((t_total, t_rebuild, int(n.value), [int(v) for v in lm.last["map_incremental"]]))
        steps.append([round(v, 3) for v in lm.last.get("t_ms", (0, 0, 0))])
        search.append((round(ms.value, 3), int(nl.value), int(nfar.value)))
    # first scan pays one-time allocations; report the median of the rest
    tt = np.median([r[0] for r in rows[1:]])
    tr = np.median([r[1] for r in rows[1:]])
    print(json.dumps({"bench": "live_mapping_per_scan", "map_points": n_map, "scan_points": n_scan,
                      "ms_fov_ikf4_map_incremental": tt, "ms_index_rebuild": tr,
                      "ms_per_scan": tt + tr, "ms_index_rebuild_each": [round(r[1], 3) for r in rows],
                      "map_size_after": rows[-1][2],
                      "map_incremental_counts_last": rows[-1][3],
                      "ms_fov_update_mapinc_each": steps,
                      "search_ms_launches_farq_each": search}), flush=True)


def chain(n_map, n_raw, frames_n=8):
    """Live laserMapping with a realistic prior: the C2-size map, raw scans
    rendered along a street with per-point time (100 ms sweep), 200 Hz IMU;
    per scan ImuProcess forward propagation (P carried, no reset) +
    undistortion + downSizeFilterSurf on the device, lasermap_fov_segment,
    the reference-flow update (maximum_iter 4), map_incremental; the index
    rebuild runs inside the next scan's first search (timed inside the
    update).  Host wall clock per stage (each stage synchronises), HIP events
    on the search launches, medians over scans 2.."""
    from agi_lidar_slam_amd import _lib as L, synth
    from agi_lidar_slam_amd.esekf import StateIkfom
    from agi_lidar_slam_amd.imu import ImuProcess, MeasureGroup
    from agi_lidar_slam_amd.mapping import LaserMapping
    import test_gpu_chain as TC
    seed = 20261015
    mp, _ = synth.make_problem(n_map, 100000, cache_dir="/tmp/slio_cache")
    seq = TC.make_sequence(seed, n_map, frames_n, n_raw, 0.5)
    lib = L.load()
    lm = LaserMapping(filter_size_map_min=0.5, cube_len=1000.0, maximum_iter=4, max_points=n_raw)
    lm.ikdtree.set_downsample_param(0.5)
    lm.ikdtree.Build(mp)
    lm.built = True
    ip = ImuProcess(mean_acc=np.array([0.0, 0.0, 1.0]), cov_gyr=TC.COV12[0:3], cov_acc=TC.COV12[3:6],
                    cov_bias_gyr=TC.COV12[6:9], cov_bias_acc=TC.COV12[9:12])
    fr0 = seq[0]["frame"]
    lm.kf.change_x(StateIkfom(pos=fr0.gt_pos.copy(), rot=fr0.gt_rot.copy(), offset_T_L_I=synth.AVIA_T_LI.copy(),
                              vel=seq[1]["v"].copy(), grav=np.array([0.0, 0.0, -9.81])))
    lm.kf.change_P(np.eye(24) * 1e-3)
    ip.last_imu_ = np.array([seq[0]["end"], 0.0, 0.0, 1.0, 0.0, 0.0, 0.0])
    ip.last_lidar_end_time_ = seq[0]["end"]
    rows = []
    for k, s in enumerate(seq[1:], start=1):
        t0 = time.perf_counter()
        meas = MeasureGroup(lidar_beg_time=s["beg"], lidar_end_time=s["end"], points=s["raw"],
                            t_ms=s["t_ms"], imu=s["imu"])
        nd = ip.undistort_downsample(meas, lm.kf, 0.5)
        t1 = time.perf_counter()
        xp = lm.kf.get_x().to_array()
        pos_lid = xp[0:3] + synth.quat_matrix(xp[3:7]) @ xp[11:14]
        lm.lasermap_fov_segment(pos_lid)
        t2 = time.perf_counter()
        lib.slio_profile(lm.kf.h, 1 << (L.SLIO_KERNEL_SEARCH + 1))
        # Nearest_Points stay on the device (map_incremental reads them there)
        lm.kf.update_iterated_dyn_share_modified(0.001, None, lm.ikdtree, None, 4, False)
        t3 = time.perf_counter()
        ms, nl = C.c_double(), C.c_int64()
        lib.slio_profile_read(lm.kf.h, L.SLIO_KERNEL_SEARCH, C.byref(ms), C.byref(nl))
        lib.slio_profile(lm.kf.h, 0)
        nfar = C.c_int64()
        lib.slio_far_queries(lm.kf.h, C.byref(nfar))
        t4 = time.perf_counter()
        cnt = lm.kf.map_incremental(lm.ikdtree, 0.5, True)
        t5 = time.perf_counter()
        st = lm.kf.last_stats
        xg = lm.kf.get_x().to_array()
        rows.append(dict(scan=k, down=int(nd), ms_imu_undistort_voxel=(t1 - t0) * 1e3,
                         ms_fov=(t2 - t1) * 1e3, ms_update_incl_rebuild=(t3 - t2) * 1e3,
                         ms_map_incremental=(t5 - t4) * 1e3, passes=int(st.passes), searches=int(st.searches),
                         launch_ms=[round(ms.value, 3), int(nl.value)], far=int(nfar.value),
                         err_m=float(np.abs(xg[0:3] - s["frame"].gt_pos).max()),
                         added=[int(v) for v in cnt]))
    keys = ["ms_imu_undistort_voxel", "ms_fov", "ms_update_incl_rebuild", "ms_map_incremental"]
    med = {k_: float(np.median([r[k_] for r in rows[1:]])) for k_ in keys}
    print(json.dumps({"bench": "live_chain_per_scan", "map_points": n_map, "raw_points": n_raw,
                      "median": med, "ms_per_scan_mapping": med["ms_fov"] + med["ms_update_incl_rebuild"]
                      + med["ms_map_incremental"], "ms_per_scan_all": sum(med.values()), "scans": rows}),
          flush=True)
    lm.kf.close()
    lm.ikdtree.close()


def preproc(n_raw):
    from agi_lidar_slam_amd.esekf import Esekf, StateIkfom
    from agi_lidar_slam_amd.imu import ImuProcess, MeasureGroup
    from imu_case import make_case
    cs = make_case(0, False, n=n_raw)
    kf = Esekf(max_points=n_raw)

    def one():
        kf.change_x(StateIkfom.from_array(cs["state"]))
        kf.change_P(cs["P"])
        ip = ImuProcess(mean_acc=np.array([0.3, 0.1, 1.02]), last_imu_=cs["imu"][0],
                        acc_s_last=cs["acc_s_last"].copy(), angvel_last=cs["angvel_last"].copy(),
                        last_lidar_end_time_=cs["last_end"])
        meas = MeasureGroup(cs["beg"], cs["end"], cs["pts"], cs["t"], cs["imu"][1:])
        return ip.undistort_downsample(meas, kf, 0.5)
    one()
    ms, nd = t_ms(one, 10)
    print(json.dumps({"bench": "undistort_voxel_per_scan", "raw_points": n_raw, "down_points": int(nd),
                      "ms_per_scan_incl_h2d": ms}), flush=True)
    kf.close()


def s2m():
    from agi_lidar_slam_amd import synth
    from agi_lidar_slam_amd.lio_sam import ScanToMap
    pr = synth.make_s2m_problem()
    s = ScanToMap(max_points=60000)
    s.set_maps(pr["corner_map"], pr["surf_map"])
    s.set_scan(pr["corner_scan"], pr["surf_scan"])
    tf = pr["tf"].copy()

    def it():
        s.corner_optimization(tf)
        s.surf_optimization(tf)
        return s.normal_equations(tf)
    it()
    ms, r = t_ms(it, 20)
    print(json.dumps({"bench": "lio_sam_s2m_iteration", "corner_points": int(pr["corner_scan"].shape[0]),
                      "surf_points": int(pr["surf_scan"].shape[0]), "ms_per_iteration": ms}), flush=True)
    s.close()


if __name__ == "__main__":
    what = sys.argv[1:] or ["mapping", "preproc", "s2m"]
    if "mapping" in what:
        mapping(10_000_000, 100_000)
    if "chain" in what:
        chain(10_000_000, int(os.environ.get("CHAIN_RAW", "100000")))
    if "preproc" in what:
        preproc(200_000)
    if "s2m" in what:
        s2m()
