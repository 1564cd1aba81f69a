"""GPU parity of the LIO-SAM scan-to-map core:
cornerOptimization / surfOptimization coefficients bit-exact vs the oracle
(oracle/lio_s2m_oracle.cpp) given the same transform, the LMOptimization
normal equations to fp32 rounding, and the whole scan2MapOptimization
converging to the ground-truth pose.  Parity unpinned: OpenCV / Eigen / PCL
are absent, their algorithms are restated (cv::eigen as OpenCV's Jacobi,
ColPivHouseholderQR, pcl::getTransformation)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_parity import L  # noqa: E402,F401

pytestmark = pytest.mark.gpu


def lidar_pose(fr):
    from agi_lidar_slam_amd import synth
    return synth.s2m_lidar_pose(fr)


@pytest.fixture(scope="module")
def problem():
    from agi_lidar_slam_amd import synth
    return synth.make_s2m_problem()


@pytest.mark.parametrize("kind", [0, 1])
def test_coeffs_bitexact(L, oracle_mod, problem, kind):
    from agi_lidar_slam_amd.lio_sam import ScanToMap
    s2m = ScanToMap(max_points=60000)
    try:
        s2m.set_maps(problem["corner_map"], problem["surf_map"])
        s2m.set_scan(problem["corner_scan"], problem["surf_scan"])
        rng = np.random.default_rng(kind)
        tf = problem["tf"] + np.concatenate([rng.uniform(-0.01, 0.01, 3), rng.uniform(-0.1, 0.1, 3)]).astype(np.float32)
        h = s2m.hc if kind == 0 else s2m.hs
        scan = problem["corner_scan"] if kind == 0 else problem["surf_scan"]
        mp = problem["corner_map"] if kind == 0 else problem["surf_map"]
        nsel = s2m.corner_optimization(tf) if kind == 0 else s2m.surf_optimization(tf)
        coeff = np.zeros((scan.shape[0], 4), np.float32)
        sel = np.zeros(scan.shape[0], np.uint8)
        L.check(L.load().slio_s2m_get_coeffs(h, L.fptr(coeff), L.u8ptr(sel)), "get")
        world = oracle_mod.s2m_transform(tf, scan)
        idx, sqd = oracle_mod.Tree(mp).knn(world, 5)
        rc, rs = oracle_mod.s2m_coeffs(kind, world, mp, idx, sqd)
        np.testing.assert_array_equal(sel, rs)
        np.testing.assert_array_equal(coeff, rc)
        assert nsel == int(rs.sum()) > (20 if kind == 0 else 1000)
    finally:
        s2m.close()


def test_normal_equations_and_convergence(L, oracle_mod, problem):
    from agi_lidar_slam_amd.lio_sam import ScanToMap
    s2m = ScanToMap(max_points=60000)
    try:
        s2m.set_maps(problem["corner_map"], problem["surf_map"])
        s2m.set_scan(problem["corner_scan"], problem["surf_scan"])
        tf0 = problem["tf"] + np.array([0.005, -0.004, 0.01, 0.15, -0.1, 0.05], np.float32)
        s2m.corner_optimization(tf0)
        s2m.surf_optimization(tf0)
        AtA, AtB, n = s2m.normal_equations(tf0)
        clouds = []
        for kind, h, scan in ((0, s2m.hc, problem["corner_scan"]), (1, s2m.hs, problem["surf_scan"])):
            coeff = np.zeros((scan.shape[0], 4), np.float32)
            sel = np.zeros(scan.shape[0], np.uint8)
            L.check(L.load().slio_s2m_get_coeffs(h, L.fptr(coeff), L.u8ptr(sel)), "get")
            clouds.append((scan, coeff, sel))
        rA, rB, rn = oracle_mod.s2m_normal_equations(tf0, clouds)
        assert n == rn
        np.testing.assert_allclose(AtA.reshape(6, 6), rA, rtol=2e-6, atol=1e-6 * np.abs(rA).max())
        np.testing.assert_allclose(AtB, rB, rtol=2e-6, atol=1e-6 * np.abs(rB).max())
        tf = s2m.scan2MapOptimization(tf0)
        err_t = np.abs(tf[3:] - problem["tf"][3:]).max()
        err_r = np.abs(tf[:3] - problem["tf"][:3]).max()
        print(f"scan2MapOptimization: {s2m.iterations} iterations, |dt| {err_t:.4f} m, |dr| {err_r:.5f} rad, "
              f"degenerate {s2m.isDegenerate.value}")
        assert err_t < 0.05 and err_r < 0.003
    finally:
        s2m.close()
