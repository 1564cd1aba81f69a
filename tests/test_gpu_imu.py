"""GPU parity of the scan undistortion: ImuProcess::
UndistortPcl's per-point back-propagation (IMU_Processing.hpp:348-401) on the
device vs the oracle's restatement (oracle/imu_oracle.cpp).  The device's
SO3 exp evaluates sin/cos by a Taylor series for small angles (the oracle:
libm, like Sophus), so the double chains can differ in the last bits; the
float results are held to 1e-5 m and are bit-equal for nearly every point."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from imu_case import make_case  # noqa: E402
from test_gpu_parity import L  # noqa: E402,F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,first_late,presorted", [(0, False, False), (1, True, False), (2, False, True)])
def test_undistort_vs_oracle(L, oracle_mod, seed, first_late, presorted):
    """presorted: the points arrive in time order (a driver's firing order),
    so the device skips its stable time sort (the identity then)."""
    from agi_lidar_slam_amd.esekf import Esekf, StateIkfom
    from agi_lidar_slam_amd.imu import ImuProcess, MeasureGroup
    cs = make_case(seed, first_late)
    if presorted:
        order = np.argsort(cs["t"], kind="stable")
        cs["pts"], cs["t"] = np.ascontiguousarray(cs["pts"][order]), np.ascontiguousarray(cs["t"][order])
    else:
        assert (np.diff(cs["t"]) < 0).any()   # the sort path
    ref = oracle_mod.imu_undistort(cs["imu"], cs["beg"], cs["end"], cs["last_end"], cs["mean_acc_norm"],
                                   cs["cov12"], cs["acc_s_last"], cs["angvel_last"], cs["state"], cs["P"],
                                   cs["pts"], cs["t"])
    kf = Esekf(max_points=cs["pts"].shape[0])
    try:
        kf.change_x(StateIkfom.from_array(cs["state"]))
        kf.change_P(cs["P"])
        ip = ImuProcess(mean_acc=np.array([0.3, 0.1, 1.02]), cov_gyr=cs["cov12"][0:3], cov_acc=cs["cov12"][3:6],
                        cov_bias_gyr=cs["cov12"][6:9], cov_bias_acc=cs["cov12"][9:12],
                        last_imu_=cs["imu"][0], acc_s_last=cs["acc_s_last"].copy(),
                        angvel_last=cs["angvel_last"].copy(), last_lidar_end_time_=cs["last_end"])
        meas = MeasureGroup(lidar_beg_time=cs["beg"], lidar_end_time=cs["end"], points=cs["pts"], t_ms=cs["t"],
                            imu=cs["imu"][1:])
        pts, t = ip.UndistortPcl(meas, kf)
        np.testing.assert_array_equal(t, ref["t_ms"])
        np.testing.assert_allclose(kf.get_x().to_array(), ref["state"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(pts, ref["points"], rtol=0, atol=1e-5)
        exact = (pts == ref["points"]).all(axis=1).mean()
        moved = (np.abs(pts - cs["pts"][np.argsort(cs["t"], kind="stable")]) > 1e-4).any(axis=1).mean()
        print(f"seed {seed}: bit-equal points {exact:.5f}, points moved by the compensation {moved:.3f}")
        assert exact > 0.99 and moved > 0.5
        # points at t = 0 are left as they are (t / 1000 > offset 0 is false)
        z = ref["t_ms"] == 0
        if not first_late:
            assert z.sum() >= 50
            np.testing.assert_array_equal(pts[z], ref["points"][z])
        # the device pipeline: undistortion + downSizeFilterSurf into the scan
        kf.change_x(StateIkfom.from_array(cs["state"]))
        kf.change_P(cs["P"])
        ip2 = ImuProcess(mean_acc=np.array([0.3, 0.1, 1.02]), cov_gyr=cs["cov12"][0:3], cov_acc=cs["cov12"][3:6],
                         cov_bias_gyr=cs["cov12"][6:9], cov_bias_acc=cs["cov12"][9:12],
                         last_imu_=cs["imu"][0], acc_s_last=cs["acc_s_last"].copy(),
                         angvel_last=cs["angvel_last"].copy(), last_lidar_end_time_=cs["last_end"])
        nd = ip2.undistort_downsample(meas, kf, 0.5)
        down = kf.feats_down_body()
        assert down.shape == (nd, 3)
        np.testing.assert_array_equal(down, oracle_mod.voxel_grid(pts, 0.5))
    finally:
        kf.close()
