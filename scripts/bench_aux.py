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
    import test_gpu_lio_s2m as T
    from agi_lidar_slam_amd.lio_sam import ScanToMap
    pr = T.problem.__wrapped__() if hasattr(T.problem, "__wrapped__") else None
    if pr is None:
        return
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
    if "preproc" in what:
        preproc(200_000)
    if "s2m" in what:
        s2m()
