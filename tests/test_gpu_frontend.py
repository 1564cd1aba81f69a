"""GPU parity of the LIO-SAM front-end (include/slio_frontend.h) with the CPU
oracle (oracle/frontend_oracle.cpp).

Bar: range image, cell owners, startRingIndex / endRingIndex, pointColInd,
pointRange, curvature, neighbour flags, labels and cloud_corner bit-exact;
deskewed coordinates bit-exact without deskew and within 1e-5 m with it (the
rotation uses sin/cos; both sides evaluate them in double and round to float,
the test reports how many agree to the bit); cloud_surface bit-exact when both
sides start from the same cloud_info.  Run on a MI355X: pytest -m gpu
"""
import sys
import os

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_frontend_oracle import small_scan  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c3():
    from agi_lidar_slam_amd import synth
    from agi_lidar_slam_amd.frontend import imu_deskew_table
    sc = synth.make_ouster_scan()
    tb = imu_deskew_table(sc["imu_stamps"], sc["imu_gyro"], sc["time_scan_cur"], sc["time_scan_end"])
    return sc, tb


def gpu_run(sc, n_scan, horizon, tb, **kw):
    from agi_lidar_slam_amd.frontend import LioSamFrontEnd, LioSamParams
    p = LioSamParams(N_SCAN=n_scan, Horizon_SCAN=horizon, **kw)
    fe = LioSamFrontEnd(p, max_points=max(len(sc["x"]), 1))
    if tb is not None and tb[4]:
        fe.set_deskew(*tb[:4], sc["time_scan_cur"], True)
    else:
        fe.set_deskew(np.zeros(1), np.zeros(1), np.zeros(1), np.zeros(1), 0.0, False)
    fe.upload(sc["x"], sc["y"], sc["z"], sc["intensity"], sc["ring"], sc["time"])
    fe.run()
    return fe


def check_projection(fe, ref, deskew):
    rm, own = fe.range_image()
    np.testing.assert_array_equal(own, ref["cell_point"])
    np.testing.assert_array_equal(rm, ref["range_mat"])
    ci = fe.cloud_info()
    for k in ("startRingIndex", "endRingIndex", "pointColInd", "pointRange"):
        np.testing.assert_array_equal(ci[k], ref[k], err_msg=k)
    if deskew:
        d = np.abs(ci["cloud_deskewed"] - ref["cloud_deskewed"])
        assert d.max() <= 1e-5, d.max()
        exact = (d == 0).all(axis=1).mean()
        print(f"deskewed points bit-exact: {exact:.6f}")
        assert exact > 0.99
    else:
        np.testing.assert_array_equal(ci["cloud_deskewed"], ref["cloud_deskewed"])
    return ci


def check_features(fe, ci, n_scan, oracle_mod, **kw):
    ref = oracle_mod.lio_features(ci, n_scan, **kw)   # same cloud_info on both sides
    got = fe.features()
    np.testing.assert_array_equal(got["cloudCurvature"], ref["cloudCurvature"])
    np.testing.assert_array_equal(got["cloudNeighborPicked"], ref["cloudNeighborPicked"])
    np.testing.assert_array_equal(got["cloudLabel"], ref["cloudLabel"])
    np.testing.assert_array_equal(got["cloud_corner"], ref["cloud_corner"])
    np.testing.assert_array_equal(got["cloud_surface"], ref["cloud_surface"])
    return got


@pytest.mark.parametrize("deskew", [False, True])
def test_c3_ouster_bitexact(oracle_mod, c3, deskew):
    sc, tb = c3
    ref = oracle_mod.lio_project(sc, 64, 2048, tb if deskew else None)
    fe = gpu_run(sc, 64, 2048, tb if deskew else None)
    try:
        ci = check_projection(fe, ref, deskew)
        got = check_features(fe, ci, 64, oracle_mod)
        assert got["cloud_corner"].shape[0] > 100 and got["cloud_surface"].shape[0] > 1000
    finally:
        fe.close()


@pytest.mark.parametrize("seed,n_scan,horizon,ds,order", [
    (3, 8, 96, 1, "ring"), (4, 8, 96, 2, "shuffled"), (5, 6, 160, 1, "shuffled"),
    (6, 16, 1800, 1, "ring"), (7, 3, 512, 1, "reversed"),
    (9, 2, 2048, 1, "ring")])   # rings of the largest horizon (ring_vsort's 2048 keys)
def test_small_scans(oracle_mod, seed, n_scan, horizon, ds, order):
    from agi_lidar_slam_amd.frontend import imu_deskew_table
    sc = small_scan(seed, n_scan=n_scan, horizon=horizon)
    n = sc["x"].size
    perm = {"ring": np.arange(n), "shuffled": np.random.default_rng(seed).permutation(n),
            "reversed": np.arange(n)[::-1]}[order]
    sc = {k: (v[perm] if isinstance(v, np.ndarray) and v.shape[:1] == (n,) else v) for k, v in sc.items()}
    tb = imu_deskew_table(sc["imu_stamps"], sc["imu_gyro"], sc["time_scan_cur"], sc["time_scan_end"])
    ref = oracle_mod.lio_project(sc, n_scan, horizon, tb, downsample_rate=ds)
    fe = gpu_run(sc, n_scan, horizon, tb, downsampleRate=ds)
    try:
        ci = check_projection(fe, ref, True)
        check_features(fe, ci, n_scan, oracle_mod)
    finally:
        fe.close()


def test_thresholds_and_leaf(oracle_mod):
    sc = small_scan(8, n_scan=8, horizon=256)
    ref = oracle_mod.lio_project(sc, 8, 256, None, min_range=2.0, max_range=11.5)
    fe = gpu_run(sc, 8, 256, None, lidarMinRange=2.0, lidarMaxRange=11.5, edgeThreshold=0.5,
                 surfThreshold=0.3, odometrySurfLeafSize=1.5)
    try:
        ci = check_projection(fe, ref, False)
        check_features(fe, ci, 8, oracle_mod, edge_threshold=0.5, surf_threshold=0.3, leaf=1.5)
    finally:
        fe.close()


@pytest.mark.parametrize("leaf", [1e-3, 0.05])
def test_voxel_grid_overflow_and_fine_leaf(oracle_mod, leaf):
    """VoxelGrid with a leaf so fine that the ring's bounding box overflows
    PCL's index check (1e-3 m: output = input, k_fe_ring's own path) or
    nearly every point is its own voxel (0.05 m: the presorted path)."""
    sc = small_scan(10, n_scan=8, horizon=256)
    ref = oracle_mod.lio_project(sc, 8, 256, None)
    fe = gpu_run(sc, 8, 256, None, odometrySurfLeafSize=leaf)
    try:
        ci = check_projection(fe, ref, False)
        check_features(fe, ci, 8, oracle_mod, leaf=leaf)
    finally:
        fe.close()


def test_edge_cases(oracle_mod):
    from agi_lidar_slam_amd.frontend import LioSamFrontEnd, LioSamParams
    sc = small_scan(3)
    empty = {k: (v[:0] if isinstance(v, np.ndarray) and v.shape[:1] == sc["x"].shape else v)
             for k, v in sc.items()}
    for case in (empty, {**sc, "ring": np.full_like(sc["ring"], 200)}):   # nothing / all bad rings
        ref = oracle_mod.lio_project(case, 8, 96, None)
        fe = gpu_run(case, 8, 96, None)
        try:
            assert fe.counts.n_extracted == 0 and fe.counts.n_corner == 0 and fe.counts.n_surface == 0
            ci = check_projection(fe, ref, False)
            check_features(fe, ci, 8, oracle_mod)
        finally:
            fe.close()
    # one ring only
    one = {k: (v[sc["ring"] == 2] if isinstance(v, np.ndarray) and v.shape[:1] == sc["x"].shape else v)
           for k, v in sc.items()}
    ref = oracle_mod.lio_project(one, 8, 96, None)
    fe = gpu_run(one, 8, 96, None)
    try:
        ci = check_projection(fe, ref, False)
        check_features(fe, ci, 8, oracle_mod)
    finally:
        fe.close()
    # capacity and state errors fail loudly
    fe = LioSamFrontEnd(LioSamParams(N_SCAN=8, Horizon_SCAN=96), max_points=10)
    try:
        from agi_lidar_slam_amd import _lib as L
        with pytest.raises(L.SlioError):
            fe.upload(sc["x"], sc["y"], sc["z"], sc["intensity"], sc["ring"], sc["time"])
        with pytest.raises(L.SlioError):
            fe.cloud_info()
    finally:
        fe.close()


def test_sector_variants_stress(oracle_mod):
    """The feature stage runs each sector's greedy picks once per possible
    prefix of suppression marks from the previous sector and chains the
    variants per ring (slio_lio.hip k_fe_pick / k_fe_ring).  Sparse rings
    (empty and 1-3 point sectors, marks that reach over an empty sector),
    planar stretches (dense flat picks right at sector ends) and low
    thresholds: bit-exact against the sequential oracle in every case."""
    for seed in range(24):
        rng = np.random.default_rng(100 + seed)
        horizon = int(rng.choice([96, 160, 240]))
        sc = small_scan(seed, n_scan=8, horizon=horizon, dup=0.05)
        n = sc["x"].size
        keep = rng.uniform(size=n) < rng.choice([0.04, 0.08, 0.15, 0.3, 0.6, 1.0])
        sc = {k: (v[keep] if isinstance(v, np.ndarray) and v.shape[:1] == (n,) else v) for k, v in sc.items()}
        kw = dict(edge_threshold=float(rng.choice([0.05, 0.3, 1.0])),
                  surf_threshold=float(rng.choice([0.05, 0.1, 0.5, 5.0])))
        ref = oracle_mod.lio_project(sc, 8, horizon, None)
        fe = gpu_run(sc, 8, horizon, None, edgeThreshold=kw["edge_threshold"],
                     surfThreshold=kw["surf_threshold"])
        try:
            ci = check_projection(fe, ref, False)
            check_features(fe, ci, 8, oracle_mod, **kw)
        finally:
            fe.close()
