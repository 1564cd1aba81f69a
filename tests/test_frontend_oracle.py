"""CPU tests of the LIO-SAM front-end oracle (oracle/frontend_oracle.cpp).

The C oracle is checked against a pure-Python loop restatement of
imageProjection.cpp:610-678 and featureExtraction.cpp:108-296 on small scans
(parity with the reference itself is unpinned: PCL / OpenCV / ROS are absent,
see DESIGN.md §front-end), plus the structural invariants of cloud_info.
"""
import math

import numpy as np
import pytest

from agi_lidar_slam_amd.frontend import imu_deskew_table


def small_scan(seed=3, n_scan=8, horizon=96, dup=0.15):
    """Ring-major scan with duplicate returns (collisions), out-of-range and
    out-of-ring points, shuffled within rings."""
    rng = np.random.default_rng(seed)
    rows = np.repeat(np.arange(n_scan), horizon)
    cols = np.tile(np.arange(horizon), n_scan)
    az = (cols - horizon // 2 + rng.uniform(-0.6, 0.6, rows.size)) * (2 * np.pi / horizon)
    el = np.deg2rad(-10 + rows * 20.0 / max(n_scan - 1, 1))
    # piecewise-smooth walls: kinks (corners), flat stretches, range jumps
    # (occlusions), a few near points (< lidarMinRange)
    r = 10.0 + np.abs(np.sin(3 * az + rows)) + 0.002 * rng.standard_normal(rows.size)
    r += np.where(np.sin(0.7 * az * horizon / 16 + rows) > 0.8, 3.0, 0.0)
    flat = np.sin(0.2 * az * horizon / 16 + 2 * rows) < -0.3
    r[flat] = 12.0 + 1e-4 * rng.standard_normal(flat.sum())        # planar stretches
    r[rng.uniform(size=rows.size) < 0.02] = 0.5
    d = np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], 1)
    p = d * r[:, None]
    extra = rng.uniform(size=rows.size) < dup
    p = np.concatenate([p, p[extra] * 1.01])
    rows = np.concatenate([rows, rows[extra]])
    cols = np.concatenate([cols, cols[extra]])
    ring = rows.astype(np.uint16)
    ring[rng.uniform(size=ring.size) < 0.01] = n_scan + 3            # bad ring
    t = (cols * (0.1 / horizon)).astype(np.float32)
    return dict(x=p[:, 0].astype(np.float32), y=p[:, 1].astype(np.float32),
                z=p[:, 2].astype(np.float32), intensity=rng.uniform(0, 100, ring.size).astype(np.float32),
                ring=ring, time=t, time_scan_cur=50.0, imu_stamps=np.arange(49.98, 50.2, 0.005),
                imu_gyro=np.tile([0.05, -0.02, 0.4], (44, 1)), time_scan_end=50.0 + float(t.max()))


# ------------------------------------------------------------------ pure-Python restatement
def py_project(sc, n_scan, horizon, table):
    ang_res_x = np.float32(360.0 / np.float32(horizon))
    rm = np.full((n_scan, horizon), np.finfo(np.float32).max, np.float32)
    own = np.full((n_scan, horizon), -1, np.int64)
    for i in range(sc["x"].size):
        x, y, z = np.float32(sc["x"][i]), np.float32(sc["y"][i]), np.float32(sc["z"][i])
        rg = np.sqrt(np.float32(np.float32(x * x) + np.float32(y * y)) + np.float32(z * z))
        rg = np.float32(np.sqrt(np.float32(np.float32(np.float32(x * x) + np.float32(y * y)) + np.float32(z * z))))
        if rg < np.float32(1.0) or rg > np.float32(1000.0):
            continue
        row = int(sc["ring"][i])
        if row >= n_scan:
            continue
        ha = np.float32(np.float32(np.float32(math.atan2(float(x), float(y))) * np.float32(180)) / math.pi)
        col = int(-round_half_away((float(ha) - 90.0) / float(ang_res_x)) + horizon // 2)
        if col >= horizon:
            col -= horizon
        if col < 0 or col >= horizon:
            continue
        if rm[row, col] != np.finfo(np.float32).max:
            continue
        rm[row, col] = rg
        own[row, col] = i
    return rm, own


def round_half_away(v):
    return math.floor(v + 0.5) if v >= 0 else -math.floor(-v + 0.5)


def py_features(info, n_scan, edge=1.0, surf=0.1):
    r = info["pointRange"].astype(np.float32)
    col = info["pointColInd"]
    n = r.size
    curv = np.zeros(n, np.float32)
    picked = np.ones(n, np.int32)
    sval = np.zeros(n, np.float32)
    sind = np.arange(n)
    for i in range(5, n - 5):
        d = np.float32(0)
        for k in (-5, -4, -3, -2, -1):
            d = np.float32(d + r[i + k])
        d = np.float32(d - np.float32(r[i] * np.float32(10)))
        for k in (1, 2, 3, 4, 5):
            d = np.float32(d + r[i + k])
        curv[i] = np.float32(d * d)
        picked[i] = 0
        sval[i] = curv[i]
    for i in range(5, n - 6):
        d1, d2 = r[i], r[i + 1]
        if abs(int(col[i + 1]) - int(col[i])) < 10:
            if float(np.float32(d1 - d2)) > 0.3:
                picked[i - 5:i + 1] = 1
            elif float(np.float32(d2 - d1)) > 0.3:
                picked[i + 1:i + 7] = 1
        a = float(abs(np.float32(r[i - 1] - r[i])))
        b = float(abs(np.float32(r[i + 1] - r[i])))
        if a > 0.02 * float(r[i]) and b > 0.02 * float(r[i]):
            picked[i] = 1
    picked0 = picked.copy()
    lab = np.zeros(n, np.int32)

    def suppress(ind):
        picked[ind] = 1
        for l in range(1, 6):
            if abs(int(col[ind + l]) - int(col[ind + l - 1])) > 10:
                break
            picked[ind + l] = 1
        for l in range(-1, -6, -1):
            if abs(int(col[ind + l]) - int(col[ind + l + 1])) > 10:
                break
            picked[ind + l] = 1

    corners, surf_pos = [], []
    st, en = info["startRingIndex"], info["endRingIndex"]
    for i in range(n_scan):
        for j in range(6):
            sp = int((st[i] * (6 - j) + en[i] * j) / 6)        # C++ truncation
            ep = int((st[i] * (5 - j) + en[i] * (j + 1)) / 6) - 1
            if sp >= ep:
                continue
            seg = sorted(range(sp, ep), key=lambda k: (float(sval[k]), int(sind[k])))
            v2, i2 = [sval[k] for k in seg], [sind[k] for k in seg]
            sval[sp:ep], sind[sp:ep] = v2, i2
            cnt = 0
            for k in range(ep, sp - 1, -1):
                ind = sind[k]
                if picked[ind] == 0 and curv[ind] > edge:
                    cnt += 1
                    if cnt <= 20:
                        lab[ind] = 1
                        corners.append(ind)
                    else:
                        break
                    suppress(ind)
            for k in range(sp, ep + 1):
                ind = sind[k]
                if picked[ind] == 0 and curv[ind] < surf:
                    lab[ind] = -1
                    suppress(ind)
            surf_pos += [k for k in range(sp, ep + 1) if lab[k] <= 0]
    return curv, picked0, lab, corners


# ------------------------------------------------------------------ tests
def test_imu_deskew_table():
    st = np.arange(10.0, 10.2, 0.005)
    g = np.tile([0.1, 0.0, 0.5], (st.size, 1))
    t, rx, ry, rz, ok = imu_deskew_table(st, g, 10.05, 10.15)
    assert ok and t[0] >= 10.04 - 1e-12 and t[-1] <= 10.16 + 1e-9
    np.testing.assert_allclose(rz, 0.5 * (t - t[0]), atol=1e-12)
    np.testing.assert_allclose(rx, 0.1 * (t - t[0]), atol=1e-12)
    # no IMU after the scan start -> unavailable
    assert not imu_deskew_table(st[:3], g[:3], 20.0, 20.1)[4]


@pytest.mark.parametrize("seed", [3, 4])
def test_oracle_projection_matches_python(oracle_mod, seed):
    sc = small_scan(seed)
    info = oracle_mod.lio_project(sc, 8, 96, None)
    rm, own = py_project(sc, 8, 96, None)
    np.testing.assert_array_equal(info["cell_point"], own)
    np.testing.assert_array_equal(info["range_mat"], rm)
    # first point wins: every owner is the smallest index mapping to its cell
    assert (own[own >= 0] >= 0).all()
    # cloudExtraction (imageProjection.cpp:656-678)
    cnt = (own >= 0).sum(axis=1)
    off = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    np.testing.assert_array_equal(info["startRingIndex"], off - 1 + 5)
    np.testing.assert_array_equal(info["endRingIndex"], off + cnt - 1 - 5)
    ci = np.concatenate([np.nonzero(own[r] >= 0)[0] for r in range(8)])
    np.testing.assert_array_equal(info["pointColInd"], ci)
    no = info["cloud_deskewed"]
    src = own[own >= 0]
    np.testing.assert_array_equal(no[:, 0], sc["x"][src])   # no deskew: points unchanged
    np.testing.assert_array_equal(no[:, 3], sc["intensity"][src])


def test_oracle_deskew_rotates_about_first_point(oracle_mod):
    sc = small_scan(5)
    tb = imu_deskew_table(sc["imu_stamps"], sc["imu_gyro"], sc["time_scan_cur"], sc["time_scan_end"])
    assert tb[4]
    a = oracle_mod.lio_project(sc, 8, 96, tb)
    b = oracle_mod.lio_project(sc, 8, 96, None)
    np.testing.assert_array_equal(a["pointRange"], b["pointRange"])  # range from the raw point
    pa, pb = a["cloud_deskewed"][:, :3], b["cloud_deskewed"][:, :3]
    # a rotation: norms kept, points moved
    np.testing.assert_allclose(np.linalg.norm(pa, axis=1), np.linalg.norm(pb, axis=1), rtol=2e-6)
    assert np.abs(pa - pb).max() > 1e-3


@pytest.mark.parametrize("seed", [3, 6])
def test_oracle_features_match_python(oracle_mod, seed):
    sc = small_scan(seed, n_scan=6, horizon=160)
    info = oracle_mod.lio_project(sc, 6, 160, None)
    fe = oracle_mod.lio_features(info, 6)
    curv, picked0, lab, corners = py_features(info, 6)
    np.testing.assert_array_equal(fe["cloudCurvature"], curv)
    np.testing.assert_array_equal(fe["cloudNeighborPicked"], picked0)
    np.testing.assert_array_equal(fe["cloudLabel"], lab)
    np.testing.assert_array_equal(fe["cloud_corner"], info["cloud_deskewed"][corners])
    assert (lab == 1).sum() > 0 and (lab == -1).sum() > 0


def test_oracle_voxel_grid_properties(oracle_mod):
    sc = small_scan(7, n_scan=4, horizon=200)
    info = oracle_mod.lio_project(sc, 4, 200, None)
    for leaf in (0.4, 2.0):
        fe = oracle_mod.lio_features(info, 4, leaf=leaf)
        su = fe["cloud_surface"]
        lab = fe["cloudLabel"]
        n_in = sum(((lab[s:e + 1] <= 0).sum()) for s, e in zip(info["startRingIndex"], info["endRingIndex"]) if e > s)
        assert 0 < su.shape[0] <= n_in
        # a larger leaf never yields more centroids
        if leaf == 2.0:
            assert su.shape[0] <= prev
        prev = su.shape[0]


def test_oracle_empty_and_tiny(oracle_mod):
    sc = small_scan(3)
    z = {k: (v[:0] if isinstance(v, np.ndarray) and v.shape[:1] == sc["x"].shape else v) for k, v in sc.items()}
    info = oracle_mod.lio_project(z, 8, 96, None)
    assert info["pointRange"].size == 0
    np.testing.assert_array_equal(info["startRingIndex"], np.full(8, 4))
    np.testing.assert_array_equal(info["endRingIndex"], np.full(8, -6))
    fe = oracle_mod.lio_features(info, 8)
    assert fe["cloud_corner"].shape[0] == 0 and fe["cloud_surface"].shape[0] == 0


def test_c3_reference_sort_ties(oracle_mod):
    """The reference sorts each sector with std::sort(by_value) on the value
    alone (featureExtraction.cpp:16-20, 201-202), so equal smoothness values
    come out in libstdc++ introsort's order; the device and the oracle break
    ties by point index.  On C3 (64 x 2048 Ouster scan) 150 keys share their
    value with another key of the same sector, and the reference's own
    std::sort call yields the identical labels, corners and surface cloud."""
    from agi_lidar_slam_amd import synth

    sc = synth.make_ouster_scan()
    tb = imu_deskew_table(sc["imu_stamps"], sc["imu_gyro"], sc["time_scan_cur"], sc["time_scan_end"])
    info = oracle_mod.lio_project(sc, 64, 2048, tb)
    by_index = oracle_mod.lio_features(info, 64)
    by_ref = oracle_mod.lio_features(info, 64, std_sort_ties=True)
    assert by_index["ties"] == by_ref["ties"] > 0
    np.testing.assert_array_equal(by_index["cloudLabel"], by_ref["cloudLabel"])
    np.testing.assert_array_equal(by_index["cloud_corner"], by_ref["cloud_corner"])
    np.testing.assert_array_equal(by_index["cloud_surface"], by_ref["cloud_surface"])
