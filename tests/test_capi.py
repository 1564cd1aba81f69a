"""CPU tests of the C-ABI boundary: the library loads, exports every symbol
include/*.h declares, and its host-only logic is right.  No GPU compute."""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest

import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*(slio_[a-z0-9_]+)\s*\(",
                             txt, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    from agi_lidar_slam_amd import build, _lib
    build.build()
    return _lib.load()


def test_header_declares_core_entry_points():
    names = declared_functions()
    for n in ["slio_create", "slio_map_upload", "slio_scan_upload", "slio_iterate",
              "slio_get_neighbors", "slio_ikf_update", "slio_destroy"]:
        assert n in names


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_bindings_cover_header():
    from agi_lidar_slam_amd import _lib
    missing = [n for n in declared_functions() if n not in _lib.SIGNATURES]
    assert not missing, missing


def test_params_default(lib):
    from agi_lidar_slam_amd import _lib as L
    p = L.SlioParams()
    assert lib.slio_params_default(C.byref(p)) == 0
    assert p.max_points == 100000 and p.nranks == 1
    assert abs(p.plane_threshold - 0.1) < 1e-7 and p.max_match_sqd == 5.0
    assert p.far_query_margin == 0.0 and p.search_radius == 0.0
    assert p.grid_cell == 0.0   # auto edge (1.0 m, 1.25 m past 2^27 cells)


def test_bad_arguments_fail_loudly(lib):
    from agi_lidar_slam_amd import _lib as L
    h = C.c_void_p()
    assert lib.slio_create(None, None) == -1
    p = L.SlioParams()
    lib.slio_params_default(C.byref(p))
    p.nranks = 3
    assert lib.slio_create(C.byref(h), C.byref(p)) == -1
    assert b"nranks" in lib.slio_last_error()
    p.nranks = 1
    p.far_query_margin = -1.0
    assert lib.slio_create(C.byref(h), C.byref(p)) == -1
    assert b"far_query_margin" in lib.slio_last_error()
    assert lib.slio_iterate_async(None, None, 1, 0, None) == -1
    # front-end C-ABI (include/slio_frontend.h): argument checks before any device call
    lp = L.SlioLioParams()
    assert lib.slio_lio_params_default(C.byref(lp)) == 0
    assert (lp.n_scan, lp.horizon_scan, lp.downsample_rate) == (16, 1800, 1)
    assert abs(lp.surf_leaf_size - 0.4) < 1e-7 and lp.edge_threshold == 1.0
    assert lib.slio_lio_create(None, None) == -1
    lp.n_scan = 0
    assert lib.slio_lio_create(C.byref(h), C.byref(lp)) == -1
    assert b"n_scan" in lib.slio_last_error()
    assert lib.slio_lio_run_async(None) == -1
    assert lib.slio_lio_destroy(None) == 0
    gp = L.SlioLegoParams()
    assert lib.slio_lego_params_default(C.byref(gp)) == 0
    assert (gp.n_scan, gp.horizon_scan, gp.ground_scan_ind) == (16, 1800, 7)
    assert (gp.segment_valid_point_num, gp.segment_valid_line_num) == (5, 3)
    assert abs(gp.ang_bottom - 15.1) < 1e-6 and abs(gp.segment_theta - 1.0472) < 1e-7
    assert lib.slio_lego_create(None, None) == -1
    gp.ground_scan_ind = 16
    assert lib.slio_lego_create(C.byref(h), C.byref(gp)) == -1
    assert b"ground_scan_ind" in lib.slio_last_error()
    assert lib.slio_lego_run_async(None) == -1
    assert lib.slio_lego_set_imu(None, None) == -1
    assert lib.slio_lego_destroy(None) == 0


def test_reduce_super_matches_python_tree(lib):
    from agi_lidar_slam_amd import _lib as L
    import tree_model as shard
    rng = np.random.default_rng(0)
    sup = rng.normal(size=(8, 91))
    sup[:, 90] = rng.integers(0, 1000, 8)
    HTH = np.zeros(78)
    HTh = np.zeros(12)
    m = C.c_int64()
    assert lib.slio_reduce_super(L.dptr(np.ascontiguousarray(sup)), L.dptr(HTH), L.dptr(HTh),
                                 C.byref(m)) == 0
    a, b, mm = shard.reduce_super(sup)
    np.testing.assert_array_equal(HTH, a)
    np.testing.assert_array_equal(HTh, b)
    assert m.value == mm


def _rotvec_to_quat(v):
    th = np.linalg.norm(v)
    if th == 0:
        return np.array([1.0, 0, 0, 0])
    return np.concatenate([[np.cos(th / 2)], np.sin(th / 2) * v / th])


def test_state_boxplus_boxminus(lib):
    """esekfom.hpp:59-73 / 236-258 on the host side of the boundary."""
    from agi_lidar_slam_amd.esekf import StateIkfom
    from agi_lidar_slam_amd import _lib as L
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(5)
    for _ in range(20):
        x = StateIkfom(pos=rng.normal(size=3), rot=_rotvec_to_quat(rng.normal(size=3)),
                       offset_R_L_I=_rotvec_to_quat(0.1 * rng.normal(size=3)),
                       offset_T_L_I=rng.normal(size=3), vel=rng.normal(size=3),
                       bg=rng.normal(size=3), ba=rng.normal(size=3), grav=rng.normal(size=3))
        dx = 0.3 * rng.normal(size=24)
        xc, out = x.to_c(), L.SlioState()
        assert lib.slio_state_boxplus(C.byref(xc), L.dptr(dx), C.byref(out)) == 0
        y = StateIkfom.from_c(out)
        # rot = rot * exp(dtheta): compare against scipy
        r_ref = Rotation.from_quat(np.r_[x.rot[1:], x.rot[0]]) * Rotation.from_rotvec(dx[3:6])
        q = r_ref.as_quat()
        q = np.r_[q[3], q[:3]]
        assert min(np.abs(q - y.rot).max(), np.abs(q + y.rot).max()) < 1e-12
        np.testing.assert_allclose(y.pos, x.pos + dx[0:3], atol=1e-15)
        np.testing.assert_allclose(y.grav, x.grav + dx[21:24], atol=1e-15)
        d = np.zeros(24)
        yc = y.to_c()
        assert lib.slio_state_boxminus(C.byref(yc), C.byref(xc), L.dptr(d)) == 0
        np.testing.assert_allclose(d, dx, atol=1e-9)


def test_library_built_from_these_sources(lib):
    """slio_build_id is the digest of the sources the library was compiled
    from; a prebuilt library that does not match the tree is caught here and
    by __graft_entry__.build()."""
    from agi_lidar_slam_amd import build
    assert lib.slio_build_id().decode() == build.source_hash()


def test_s2m_lm_step_singular_is_a_zero_step(lib):
    """LIO-SAM LMOptimization (mapOptmization.cpp:1620): cv::solve(DECOMP_QR)
    gives up on an R diagonal below 10 * FLT_EPSILON, zeroes matX, and the
    caller ignores the result -- a zero step that reads as converged, not an
    abort.  A well-conditioned system still solves."""
    from agi_lidar_slam_amd import _lib as L
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32)
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))
    for AtA in (np.zeros((6, 6)), np.diag([1.0, 1, 1, 1, 1, 0]),
                np.diag([1.0, 1, 1, 1, 1, 1e-9])):
        AtA, AtB = f32(AtA), f32(np.arange(1, 7))
        tf = f32(np.array([0.1, 0.2, 0.3, 1.0, 2.0, 3.0]))
        tf0 = tf.copy()
        deg, conv = C.c_int(0), C.c_int(0)
        matP = f32(np.zeros((6, 6)))
        rc = lib.slio_s2m_lm_step(fp(AtA), fp(AtB), 100, 1, fp(tf), C.byref(deg), fp(matP), C.byref(conv))
        assert rc == 0, L.last_error() if hasattr(L, "last_error") else rc
        np.testing.assert_array_equal(tf, tf0)
        assert conv.value == 1
    # regular system: transform moves by the solution
    A = np.diag([1e3, 2e3, 3e3, 4e3, 5e3, 6e3])
    b = np.array([1.0, 2, 3, 4, 5, 6]) * 1e-3
    AtA, AtB = f32(A), f32(b)
    tf = f32(np.zeros(6))
    deg, conv = C.c_int(0), C.c_int(0)
    matP = f32(np.zeros((6, 6)))
    assert lib.slio_s2m_lm_step(fp(AtA), fp(AtB), 100, 1, fp(tf), C.byref(deg), fp(matP), C.byref(conv)) == 0
    np.testing.assert_allclose(tf, np.linalg.solve(A, b), rtol=1e-5)
