"""CPU tests: pin the oracle against the committed golden vectors and
independent implementations (no GPU needed)."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_knn_matches_golden(oracle_mod):
    z = np.load(os.path.join(GOLD, "knn_golden.npz"))
    T = oracle_mod.Tree(z["map"])
    idx, sqd = T.knn(z["query"], 5, threads=4)
    np.testing.assert_array_equal(idx, z["idx"])
    np.testing.assert_array_equal(sqd, z["sqd"])


def test_knn_sqd_is_reference_float_formula(oracle_mod):
    z = np.load(os.path.join(GOLD, "knn_golden.npz"))
    T = oracle_mod.Tree(z["map"])
    q = z["query"][:500]
    idx, sqd = T.knn(q, 5, threads=2)
    p = z["map"][idx]
    d = q[:, None, :] - p
    ref = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    np.testing.assert_array_equal(sqd, ref.astype(np.float32))
    assert np.all(np.diff(sqd, axis=1) >= 0)


def test_knn_small_and_empty_maps(oracle_mod):
    mp = np.array([[0, 0, 0], [1, 0, 0], [0, 2, 0]], np.float32)
    T = oracle_mod.Tree(mp)
    idx, sqd = T.knn(np.array([[0.1, 0, 0]], np.float32), 5)
    assert list(idx[0, :3]) == [0, 1, 2] and list(idx[0, 3:]) == [-1, -1]
    assert np.isinf(sqd[0, 3:]).all()


def test_knn_random_vs_scipy(oracle_mod):
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(3)
    mp = rng.uniform(-50, 50, (30000, 3)).astype(np.float32)
    mp[:, 2] *= 0.05
    q = rng.uniform(-60, 60, (2000, 3)).astype(np.float32)
    T = oracle_mod.Tree(mp)
    idx, sqd = T.knn(q, 5)
    _, ii = cKDTree(mp.astype(np.float64)).query(q.astype(np.float64), 5)
    # compare as sets of distances (float64 ranking may swap near-equal f32 pairs)
    d = q[:, None, :] - mp[ii]
    ref = np.sort((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2], 1)
    np.testing.assert_array_equal(sqd, ref)


def test_esti_plane_vs_lstsq(oracle_mod):
    z = np.load(os.path.join(GOLD, "plane_golden.npz"))
    n_ok = 0
    for nb, pl, ok in zip(z["nb"], z["plane"], z["ok"]):
        got_ok, got = oracle_mod.esti_plane(nb, 0.1)
        assert got_ok == bool(ok)
        # same plane up to float32 conditioning of the 5x3 system
        np.testing.assert_allclose(got[:3], pl[:3], atol=2e-4)
        np.testing.assert_allclose(got[3], pl[3], rtol=2e-3, atol=2e-3)
        n_ok += got_ok
    assert n_ok > 1000


def test_esti_plane_degenerate(oracle_mod):
    # collinear neighbours: rank-deficient A (nonzero_pivots < 3 path)
    nb = np.array([[0, 0, 1], [1, 0, 1], [2, 0, 1], [3, 0, 1], [4, 0, 1]], np.float32)
    ok, pl = oracle_mod.esti_plane(nb, 0.1)
    assert ok
    np.testing.assert_allclose(np.abs(pl[:3]), [0, 0, 1], atol=1e-6)
    np.testing.assert_allclose(pl[3], -np.sign(pl[2]) * 1.0, atol=1e-6)


def test_ikf_oracle_converges_and_control_flow(oracle_mod):
    from agi_lidar_slam_amd import synth
    mp, fr = synth.make_problem(200000, 20000, pattern="vlp16")
    T = oracle_mod.Tree(mp)
    st = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9),
                         [0, 0, -9.81]])
    s2, P2, stats, idx, sqd, sel = oracle_mod.ikf_update(T, fr.body, st, np.eye(24),
                                                         maximum_iter=3, mode=0)
    passes, searches, valid, converged, m = stats
    assert 2 <= passes <= 4 and valid == passes and searches >= 1
    ang = 2 * np.arccos(min(1.0, abs(np.dot(s2[3:7], fr.gt_rot))))
    ang0 = 2 * np.arccos(min(1.0, abs(np.dot(fr.init_rot, fr.gt_rot))))
    assert ang < 0.25 * ang0
    assert np.linalg.norm(s2[:3] - fr.gt_pos) < np.linalg.norm(st[:3] - fr.gt_pos)
    # P = (I - KH) P equals (H^T H / R + P^-1)^-1: symmetric up to rounding, SPD
    assert np.abs(P2 - P2.T).max() < 1e-6 * np.abs(P2).max() + 1e-6
    assert np.all(np.linalg.eigvalsh(0.5 * (P2 + P2.T)) > -1e-8)
    # reference K (24 x m) and reduced K*h / K*H forms agree
    s3, P3, *_ = oracle_mod.ikf_update(T, fr.body, st, np.eye(24), maximum_iter=3, mode=0,
                                       reference_gain=0)
    np.testing.assert_allclose(s3, s2, atol=1e-9)
    np.testing.assert_allclose(P3, P2, atol=1e-6 * np.abs(P2).max())


def test_pass_gates(oracle_mod):
    from agi_lidar_slam_amd import synth
    mp, fr = synth.make_problem(200000, 20000, pattern="avia")
    T = oracle_mod.Tree(mp)
    st = np.concatenate([fr.gt_pos, fr.gt_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9),
                         [0, 0, -9.81]])
    ps = oracle_mod.PassState(fr.body.shape[0])
    out = oracle_mod.h_pass(T, st, fr.body, ps, True)
    m = int(out[90])
    assert m == int(ps.sel.sum()) and m > 0.5 * fr.body.shape[0]
    # selected points: finite planes, |pd2| small, 5th distance within the gate
    s = ps.sel.astype(bool)
    assert np.isfinite(ps.plane[s]).all() and np.all(ps.sqd[s, 4] <= 5.0)
    assert np.all(np.abs(ps.resid[s]) < 0.5)
    # a non-search pass at the same pose keeps the selection
    sel0 = ps.sel.copy()
    out2 = oracle_mod.h_pass(T, st, fr.body, ps, False)
    np.testing.assert_array_equal(ps.sel, sel0)
    np.testing.assert_array_equal(out2, out)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("ext", [False, True])
def test_reference_gain_equals_reduced_gain(oracle_mod, mode, ext):
    """The reference's own gain formation (esekfom.hpp:311-319: K =
    K_front[:, :12] H^T / R as a 24 x m matrix, then K h and K H) against
    the H^T H / H^T h form the GPU path reduces to (reference_gain=0): the
    same control flow and neighbours, x and P equal to rounding.  Without
    extrinsic estimation within 1e-12 (x, absolute) and 1e-12 of max |P|; with
    it the 12-column system's directions that only the prior observes make
    S = P^-1 + E^T H^T H E / R ill-conditioned (kappa ~ 2e8 here), so the two
    orderings of the same sums may differ by up to u * kappa (x) and
    32 u kappa max|P| (P)."""
    from agi_lidar_slam_amd import synth
    mp, fr = synth.make_problem(200000, 20000, pattern="avia")
    T = oracle_mod.Tree(mp)
    st = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9),
                         [0, 0, -9.81]])
    P0 = np.eye(24) * 1e-2
    a = oracle_mod.ikf_update(T, fr.body, st, P0, maximum_iter=4, mode=mode, extrinsic=ext,
                              reference_gain=1, threads=8)
    b = oracle_mod.ikf_update(T, fr.body, st, P0, maximum_iter=4, mode=mode, extrinsic=ext,
                              reference_gain=0, threads=8)
    np.testing.assert_array_equal(a[2], b[2])   # passes, searches, valid, converged, m
    np.testing.assert_array_equal(a[3], b[3])   # Nearest_Points of the last search
    np.testing.assert_array_equal(a[5], b[5])   # point_selected_surf
    dx, dP, pmax = np.abs(a[0] - b[0]).max(), np.abs(a[1] - b[1]).max(), np.abs(a[1]).max()
    if not ext:
        assert dx <= 1e-12, dx
        assert dP <= 1e-12 * pmax, dP
    else:
        rows = np.zeros((fr.body.shape[0], 14))
        oracle_mod.h_pass(T, st, fr.body, oracle_mod.PassState(fr.body.shape[0]), True, extrinsic=True,
                          rows=rows)
        S = np.linalg.inv(P0)
        S[:12, :12] += rows[:, :12].T @ rows[:, :12] / 0.001
        u, kappa = 2.0 ** -52, np.linalg.cond(S)
        assert dx <= u * kappa, (dx, kappa)
        assert dP <= 32 * u * kappa * pmax, (dP, kappa)
