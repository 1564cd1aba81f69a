"""GPU parity of the LeGO-LOAM front-end (slio_lego_*, include/slio_frontend.h)
with the CPU oracle (oracle/frontend_oracle.cpp orc_lego_*).

Bar: range image, cell owners, groundMat, labelMat (component labels in the
reference's labelCount order), cloud_info and the segmented / outlier clouds
bit-exact; curvature, neighbour flags, labels and the four feature clouds
bit-exact when both sides start from the same segmented cloud; the
adjustDistortion output bit-exact without IMU and within 1e-5 m with it (the
rotation uses sin/cos evaluated in double and rounded to float on both sides;
the test reports how many points agree to the bit).  Run on a MI355X:
pytest -m gpu
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_lego_oracle import small_sweep  # noqa: E402

pytestmark = pytest.mark.gpu


def run_both(oracle_mod, sc, P, imu=None, t0=0.0, max_points=0):
    from agi_lidar_slam_amd.lego import LegoFrontEnd
    fe = LegoFrontEnd(P, max_points=max_points or max(sc["x"].size, 1))
    fe.set_imu(imu, t0)
    fe.upload(sc["x"], sc["y"], sc["z"])
    fe.run()
    ref = oracle_mod.lego_project(sc["x"], sc["y"], sc["z"], P)
    return fe, ref


def check_image(fe, ref):
    im = fe.image()
    for k in ("cell_point", "range_mat", "ground", "label"):
        np.testing.assert_array_equal(im[k], ref[k], err_msg=k)
    si = fe.seg_info()
    for k in ("orientation", "startRingIndex", "endRingIndex", "segmentedCloudGroundFlag",
              "segmentedCloudColInd", "segmentedCloudRange", "segmented_cloud", "outlier_cloud"):
        np.testing.assert_array_equal(si[k], ref[k], err_msg=k)
    return si


def check_features(oracle_mod, fe, si, P, imu=None, t0=0.0):
    ref = oracle_mod.lego_features(si, P, imu, t0)
    got = fe.features()
    d = np.abs(got["deskewed"] - ref["deskewed"])
    if imu is None:
        np.testing.assert_array_equal(got["deskewed"], ref["deskewed"])
    else:
        assert d.size == 0 or d.max() <= 1e-5, d.max()
        if d.size:
            exact = (d == 0).all(axis=1).mean()
            print(f"deskewed points bit-exact: {exact:.6f}")
            assert exact > 0.99
    for k in ("cloudCurvature", "cloudNeighborPicked", "cloudLabel"):
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    if imu is None or d.size == 0 or d.max() == 0:
        for k in ("cornerPointsSharp", "cornerPointsLessSharp", "surfPointsFlat",
                  "surfPointsLessFlat"):
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    else:
        # same selection; coordinates within the deskew tolerance
        for k in ("cornerPointsSharp", "cornerPointsLessSharp", "surfPointsFlat"):
            assert got[k].shape == ref[k].shape, k
            np.testing.assert_allclose(got[k], ref[k], atol=1e-5, err_msg=k)
        assert abs(got["surfPointsLessFlat"].shape[0] - ref["surfPointsLessFlat"].shape[0]) <= 2
    for k in ("rpy_start", "rpy_cur", "velo_from_start", "angular_from_start", "ang_last"):
        np.testing.assert_array_equal(got["imu_out"][k], ref["imu_out"][k], err_msg=k)
    assert got["imu_out"]["pointer_last_iteration"] == ref["imu_out"]["pointer_last_iteration"]
    return got


@pytest.mark.parametrize("with_imu,cc", [(False, "band"), (True, "band"), (False, "lds1"), (False, "global"),
                                         (True, "band-rows-split")])
def test_vlp16_sweep_bitexact(oracle_mod, with_imu, cc, monkeypatch):
    """cc: labelComponents in 64-column bands with a last-arriver seam merge
    (k_lego_cc_band, the default for <= 64 rows), by the one-workgroup LDS
    union-find (k_lego_cc, SLIO_LEGO_CC_LDS1) or by the global-atomic kernels
    (SLIO_LEGO_CC_GLOBAL): the same labels.  band-rows-split: the row stage as
    four launches (SLIO_LEGO_ROWS_SPLIT, the A/B baseline of k_lego_rows)."""
    if cc == "band-rows-split":
        monkeypatch.setenv("SLIO_LEGO_ROWS_SPLIT", "1")
    if cc == "global":
        monkeypatch.setenv("SLIO_LEGO_CC_GLOBAL", "1")
    if cc == "lds1":
        monkeypatch.setenv("SLIO_LEGO_CC_LDS1", "1")
    from agi_lidar_slam_amd import synth
    from agi_lidar_slam_amd.lego import LegoImu, LegoParams
    P = LegoParams()
    sw = synth.make_vlp16_sweep()
    imu = None
    if with_imu:
        imu = LegoImu()
        imu.feed(sw["imu"], sw["time_scan_cur"] + 0.15)
    fe, ref = run_both(oracle_mod, sw, P, imu, sw["time_scan_cur"])
    try:
        si = check_image(fe, ref)
        got = check_features(oracle_mod, fe, si, P, imu, sw["time_scan_cur"])
        assert got["cornerPointsSharp"].shape[0] > 20 and got["surfPointsFlat"].shape[0] > 20
        assert got["surfPointsLessFlat"].shape[0] > 1000
    finally:
        fe.close()


@pytest.mark.parametrize("cc", ["band", "lds1"])
@pytest.mark.parametrize("seed,n_scan,horizon,res_y,shuffle,dup", [
    (3, 16, 360, 2.0, False, 0.1), (4, 16, 240, 2.0, True, 0.3), (5, 32, 1024, 1.0, True, 0.05),
    (6, 64, 2048, 0.5, False, 0.0), (7, 8, 97, 4.0, False, 0.2), (9, 4, 65, 8.0, True, 0.2)])
def test_small_sweeps(oracle_mod, seed, n_scan, horizon, res_y, shuffle, dup, cc, monkeypatch):
    """Geometries beside VLP-16's, each labelComponents path: bands (default
    where it applies: <= 64 rows; 97 and 65 columns leave a narrow last band,
    the column wrap crosses a seam; 64 x 2048 is past the bands' merge table
    and takes the global kernels) or the one-workgroup LDS kernel."""
    if cc == "lds1":
        monkeypatch.setenv("SLIO_LEGO_CC_LDS1", "1")
    from agi_lidar_slam_amd.lego import LegoParams
    P = LegoParams(N_SCAN=n_scan, Horizon_SCAN=horizon, ang_res_x=360.0 / horizon, ang_res_y=res_y,
                   groundScanInd=min(7, n_scan - 1))
    sc = small_sweep(seed, n_scan=n_scan, horizon=horizon, res_y=res_y, dup=dup, shuffle=shuffle)
    fe, ref = run_both(oracle_mod, sc, P)
    try:
        si = check_image(fe, ref)
        check_features(oracle_mod, fe, si, P)
    finally:
        fe.close()


def test_params_and_repeat(oracle_mod):
    """Non-default thresholds / leaf / mount angle, and the same handle run on
    two different sweeps (no state leaks between scans)."""
    from agi_lidar_slam_amd.lego import LegoFrontEnd, LegoParams
    P = LegoParams(Horizon_SCAN=360, ang_res_x=1.0, edgeThreshold=0.3, surfThreshold=0.05,
                   leafSize=0.5, sensorMountAngle=2.0, segmentTheta=0.9, segmentValidPointNum=4,
                   segmentValidLineNum=2)
    fe = LegoFrontEnd(P, max_points=20000)
    try:
        for seed in (11, 12):
            sc = small_sweep(seed, horizon=360)
            fe.set_imu(None)
            fe.upload(sc["x"], sc["y"], sc["z"])
            fe.run()
            ref = oracle_mod.lego_project(sc["x"], sc["y"], sc["z"], P)
            si = check_image(fe, ref)
            check_features(oracle_mod, fe, si, P)
    finally:
        fe.close()


def test_edge_cases(oracle_mod):
    from agi_lidar_slam_amd import _lib as L
    from agi_lidar_slam_amd.lego import LegoFrontEnd, LegoParams
    P = LegoParams(Horizon_SCAN=360, ang_res_x=1.0)
    z = np.zeros(0, np.float32)
    one = np.ones(1, np.float32)
    up = np.full(50, 30.0, np.float32)  # all above the top ring
    for sc in ({"x": z, "y": z, "z": z}, {"x": one, "y": one, "z": one * 0},
               {"x": np.ones(50, np.float32), "y": np.ones(50, np.float32), "z": up}):
        fe, ref = run_both(oracle_mod, sc, P, max_points=64)
        try:
            si = check_image(fe, ref)
            check_features(oracle_mod, fe, si, P)
        finally:
            fe.close()
    fe = LegoFrontEnd(P, max_points=10)
    try:
        with pytest.raises(L.SlioError):
            fe.upload(np.zeros(11, np.float32), np.zeros(11, np.float32), np.zeros(11, np.float32))
        with pytest.raises(L.SlioError):
            fe.seg_info()
    finally:
        fe.close()


def test_sector_variants_stress(oracle_mod):
    """LeGO-LOAM's feature rules through the per-sector variant chain
    (k_fe_pick / k_fe_ring): thinned sweeps (empty and tiny sectors), low
    thresholds (many picks, marks at every sector end), the 4-flat cap whose
    4th pick does not suppress.  Bit-exact against the sequential oracle."""
    from agi_lidar_slam_amd.lego import LegoParams
    for seed in range(16):
        rng = np.random.default_rng(200 + seed)
        horizon = int(rng.choice([240, 360, 512]))
        P = LegoParams(N_SCAN=16, Horizon_SCAN=horizon, ang_res_x=360.0 / horizon, ang_res_y=2.0,
                       groundScanInd=7, edgeThreshold=float(rng.choice([0.05, 0.1, 0.3])),
                       surfThreshold=float(rng.choice([0.05, 0.1, 1.0])), segmentValidPointNum=3,
                       segmentValidLineNum=2)
        sc = small_sweep(seed, n_scan=16, horizon=horizon, res_y=2.0, dup=0.05, shuffle=bool(seed % 2))
        n = sc["x"].size
        keep = rng.uniform(size=n) < rng.choice([0.2, 0.4, 0.7, 1.0])
        sc = {k: (v[keep] if isinstance(v, np.ndarray) and v.shape[:1] == (n,) else v) for k, v in sc.items()}
        fe, ref = run_both(oracle_mod, sc, P)
        try:
            si = check_image(fe, ref)
            check_features(oracle_mod, fe, si, P)
        finally:
            fe.close()


def seam_sweep(horizon=1800, n_scan=16, res_y=2.0):
    """Walls all around the sensor: rings above the horizon hit a cylinder of
    20 m (rings 12-15: one component across every 64-column band seam and
    the column wrap) or of 8 m (rings 8-11, with no return every 97th column:
    ~19 components of 96 columns, most across a seam), rings below it the
    ground -- the seam merge of k_lego_cc_band decides every label."""
    cols = np.repeat(np.arange(horizon), n_scan)
    rings = np.tile(np.arange(n_scan), horizon)
    az = -(cols + 0.25) * (2 * np.pi / horizon) + np.pi
    el = np.deg2rad(-15.0 + res_y * rings)
    d = np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], 1)
    rad = np.where(rings >= 12, 20.0, 8.0)
    with np.errstate(divide="ignore"):
        t = np.where(d[:, 2] < 0, -1.7 / d[:, 2], rad / np.hypot(d[:, 0], d[:, 1]))
    keep = ~((rings >= 8) & (rings < 12) & (cols % 97 == 0))
    p = (d * t[:, None]).astype(np.float32)[keep]
    return dict(x=p[:, 0].copy(), y=p[:, 1].copy(), z=p[:, 2].copy())


def test_components_span_every_seam(oracle_mod):
    """Components that span every band seam and the column wrap, the same
    handle run 12 times: labels, sizes and the segmented cloud bit-exact
    against the oracle every time (the bands' parent / csize / rows stores
    and the last band's merge stores to the same words must not race through
    two XCDs' L2 write-backs)."""
    from agi_lidar_slam_amd.lego import LegoFrontEnd, LegoParams
    P = LegoParams()
    sc = seam_sweep()
    ref = oracle_mod.lego_project(sc["x"], sc["y"], sc["z"], P)
    fe = LegoFrontEnd(P, max_points=sc["x"].size)
    try:
        for _ in range(12):
            fe.set_imu(None)
            fe.upload(sc["x"], sc["y"], sc["z"])
            fe.run()
            si = check_image(fe, ref)
        lab = fe.image()["label"]
        assert len(np.unique(lab[(lab > 0) & (lab < 999999)])) >= 15  # the 20 m wall, the 8 m pieces
    finally:
        fe.close()
