"""CPU: the library's host forward propagation of UndistortPcl
(slio_imu_forward / slio_ikf_predict, csrc/slio_imu.cpp) against the oracle's
restatement (oracle/imu_oracle.cpp) -- IMU_Processing.hpp:253-346,
esekfom.hpp:82-95, use-ikfom.hpp:45-117.  No GPU needed: the forward pass is
host C++."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from imu_case import make_case  # noqa: E402


@pytest.mark.parametrize("seed,first_late", [(0, False), (1, True)])
def test_forward_matches_oracle(oracle_mod, seed, first_late):
    from agi_lidar_slam_amd import _lib as L
    from agi_lidar_slam_amd.esekf import StateIkfom
    cs = make_case(seed, first_late, n=1000)
    ref = oracle_mod.imu_undistort(cs["imu"], cs["beg"], cs["end"], cs["last_end"], cs["mean_acc_norm"],
                                   cs["cov12"], cs["acc_s_last"], cs["angvel_last"], cs["state"], cs["P"],
                                   cs["pts"], cs["t"])
    imu = cs["imu"]
    samples = (L.SlioImuSample * imu.shape[0])()
    for k, r in enumerate(imu):
        samples[k].t = r[0]
        samples[k].acc[:] = list(r[1:4])
        samples[k].gyr[:] = list(r[4:7])
    poses = (L.SlioImuPose * imu.shape[0])()
    npose = C.c_int()
    lle = C.c_double(cs["last_end"])
    xs = StateIkfom.from_array(cs["state"]).to_c()
    P = cs["P"].copy()
    asl, avl = cs["acc_s_last"].copy(), cs["angvel_last"].copy()
    cov = [np.ascontiguousarray(cs["cov12"][3 * k:3 * k + 3]) for k in range(4)]
    L.check(L.load().slio_imu_forward(samples, imu.shape[0], cs["beg"], cs["end"], C.byref(lle),
                                      cs["mean_acc_norm"], *(L.dptr(c) for c in cov), L.dptr(asl), L.dptr(avl),
                                      C.byref(xs), L.dptr(P), poses, imu.shape[0], C.byref(npose)), "forward")
    assert npose.value == ref["poses"].shape[0] > 10
    got = np.array([[p.offset_time, *p.acc, *p.gyr, *p.vel, *p.pos, *p.rot] for p in poses[:npose.value]])
    np.testing.assert_allclose(got, ref["poses"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(StateIkfom.from_c(xs).to_array(), ref["state"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(P, ref["P"], rtol=1e-10, atol=1e-15)
    np.testing.assert_allclose(asl, ref["acc_s_last"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(avl, ref["angvel_last"], rtol=1e-12, atol=1e-12)
    assert lle.value == ref["last_lidar_end_time"] == cs["end"]
