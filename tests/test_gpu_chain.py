"""The whole laserMapping scan chain, scan after scan, device vs oracle
(SURVEY.md §8a-1 + §8f; laserMapping.cpp:719-786, IMU_Processing.hpp:253-441):

  p_imu1->Process: the forward propagation over the scan's IMU samples
      (esekf::predict, P carried from scan to scan -- no reset) and the
      per-point undistortion        -> slio_imu_forward + the device pipeline
  downSizeFilterSurf (:737-739)     -> slio_scan_upload_undistort_voxel
  lasermap_fov_segment (:736)       -> slio_fov_segment + Delete_Point_Boxes
  update_iterated_dyn_share_modified (:772)
  map_incremental (:786)            -> slio_map_incremental

Every stage is checked against the oracle's restatement, starting each scan
from the state and covariance the device holds (oracle/imu_oracle.cpp,
voxel_grid, fov_segment, ikf_update, map_oracle.cpp): the propagated state
and covariance to 1e-12, the downsampled scan to 1e-5 m with the same size,
the updated state to the north_star tolerance (1e-4 m / 1e-5 rad), and the
maps bit-equal after every scan -- the oracle's map driven by the ORACLE's
own Nearest_Points (its own kNN of its own update), so a kNN divergence at
any scan would show up as a map difference.

The synthetic sensor drives along a street (synth.make_trajectory); its IMU
samples (200 Hz) turn at the constant rate between consecutive scan poses
and read gravity only (no acceleration in the world), the state's velocity
starts at the first displacement / 0.1 s, and every raw point is rendered at
its own time in [0, 100) ms from the pose the constant-velocity motion gives
then, so the undistortion has real work: points move by up to ~0.6 m.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_map import assert_same_map  # noqa: E402
from test_gpu_parity import L, rot_err  # noqa: E402,F401

pytestmark = pytest.mark.gpu

DT = 0.1            # scan period (s)
IMU_DT = 0.005      # 200 Hz
T0 = 1.0            # end time of scan 0
COV12 = np.array([0.1] * 3 + [0.1] * 3 + [1e-4] * 3 + [1e-4] * 3)


def rotvec_of(q):
    w, v = q[0], np.asarray(q[1:], dtype=np.float64)
    n = np.linalg.norm(v)
    if n < 1e-15:
        return 2.0 * v
    return 2.0 * np.arctan2(n, w) * v / n


def make_sequence(seed, n_map, n_frames, n_scan, step):
    """Frames + per-scan IMU samples + raw (time-distorted) points."""
    from agi_lidar_slam_amd import synth
    frames = synth.make_trajectory(seed, n_map, n_frames, n_scan, step=step)
    rng = np.random.default_rng(seed + 5)
    t_li = synth.AVIA_T_LI
    seq = []
    for k, fr in enumerate(frames):
        t_end = T0 + DT * k
        if k == 0:
            seq.append(dict(frame=fr, beg=t_end - DT, end=t_end, imu=None, raw=fr.body.copy(),
                            t_ms=np.zeros(fr.body.shape[0], np.float32)))
            continue
        prev = frames[k - 1]
        R0 = synth.quat_matrix(prev.gt_rot)
        # body-frame rate taking prev.gt_rot to fr.gt_rot in DT
        dq = synth.quat_mul(np.array([prev.gt_rot[0], *(-prev.gt_rot[1:])]), fr.gt_rot)
        w = rotvec_of(dq) / DT
        v = (fr.gt_pos - prev.gt_pos) / DT

        def rot_at(t):
            return R0 @ synth.quat_matrix(synth.quat_from_rotvec(w * (t - (t_end - DT))))

        def pos_at(t):
            return prev.gt_pos + v * (t - (t_end - DT))

        ts = np.arange(t_end - DT + IMU_DT, t_end + 1e-9, IMU_DT)
        imu = np.array([[t, *(rot_at(t).T @ np.array([0.0, 0.0, 1.0])), *w] for t in ts])
        # raw points: world point of the end-pose return, seen from the pose at its own time
        Re = synth.quat_matrix(fr.gt_rot)
        W = (fr.body.astype(np.float64) + t_li) @ Re.T + fr.gt_pos
        tau = np.sort(rng.uniform(0.0, 100.0, fr.body.shape[0])).astype(np.float32)
        tt = (t_end - DT) + tau.astype(np.float64) / 1000.0
        raw = np.empty_like(W)
        for i0 in range(0, W.shape[0], 4096):
            sl = slice(i0, i0 + 4096)
            Rt = np.stack([rot_at(t) for t in tt[sl]])
            pt = np.stack([pos_at(t) for t in tt[sl]])
            raw[sl] = np.einsum("nji,nj->ni", Rt, W[sl] - pt) - t_li
        seq.append(dict(frame=fr, beg=t_end - DT, end=t_end, imu=imu, raw=raw.astype(np.float32), t_ms=tau,
                        v=v))
    return seq


def run_chain(L, oracle_mod, seq, map_points_fn, max_points, check_every=1):
    from agi_lidar_slam_amd import synth
    from agi_lidar_slam_amd.esekf import StateIkfom
    from agi_lidar_slam_amd.imu import ImuProcess, MeasureGroup
    from agi_lidar_slam_amd.mapping import LaserMapping
    lm = LaserMapping(filter_size_map_min=0.5, cube_len=124.0, det_range=40.0, maximum_iter=4,
                      max_points=max_points)
    ip = ImuProcess(mean_acc=np.array([0.0, 0.0, 1.0]), cov_gyr=COV12[0:3], cov_acc=COV12[3:6],
                    cov_bias_gyr=COV12[6:9], cov_bias_acc=COV12[9:12])
    om = None
    omin, omax = np.zeros(3, np.float32), np.zeros(3, np.float32)
    oini = False
    fr0 = seq[0]["frame"]
    x = StateIkfom(pos=fr0.gt_pos.copy(), rot=fr0.gt_rot.copy(), offset_T_L_I=synth.AVIA_T_LI.copy(),
                   vel=seq[1]["v"].copy(), grav=np.array([0.0, 0.0, -9.81]))
    lm.kf.change_x(x)
    lm.kf.change_P(np.eye(24) * 1e-3)
    report = []
    try:
        for k, s in enumerate(seq):
            if k == 0:
                # the first scan builds the map (laserMapping.cpp:750-765); the
                # IMU process starts here (its last sample and lidar end time)
                ip.last_imu_ = np.array([s["end"], 0.0, 0.0, 1.0, 0.0, 0.0, 0.0])
                ip.last_lidar_end_time_ = s["end"]
                st = lm.kf.get_x().to_array()
                pos_lid = st[0:3] + synth.quat_matrix(st[3:7]) @ st[11:14]
                lm.lasermap_fov_segment(pos_lid)
                down = oracle_mod.voxel_grid(s["raw"], 0.5)
                lm.ikdtree.set_downsample_param(0.5)
                lm.ikdtree.Build(oracle_mod.body_to_world_mat(st, down))
                lm.built = True
                oini, _ = oracle_mod.fov_segment(pos_lid, omin, omax, oini, cube_len=124.0, det_range=40.0)
                om = oracle_mod.Map(oracle_mod.body_to_world_mat(st, down))
                assert_same_map(L, lm.ikdtree.h, om)
                continue
            # ---- p_imu1->Process: forward propagation + undistortion + downsampling
            x_before = lm.kf.get_x().to_array()
            P_before = lm.kf.get_P().copy()
            imu_in = np.concatenate([ip.last_imu_[None], s["imu"]])
            ref = oracle_mod.imu_undistort(imu_in, s["beg"], s["end"], ip.last_lidar_end_time_, 1.0, COV12,
                                           ip.acc_s_last, ip.angvel_last, x_before, P_before, s["raw"],
                                           s["t_ms"])
            meas = MeasureGroup(lidar_beg_time=s["beg"], lidar_end_time=s["end"], points=s["raw"],
                                t_ms=s["t_ms"], imu=s["imu"])
            nd = ip.undistort_downsample(meas, lm.kf, 0.5)
            x_prop = lm.kf.get_x().to_array()
            P_prop = lm.kf.get_P().copy()
            np.testing.assert_allclose(x_prop, ref["state"], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(P_prop, ref["P"], rtol=1e-10, atol=1e-14)
            down = lm.kf.feats_down_body()
            oref_down = oracle_mod.voxel_grid(ref["points"], 0.5)
            assert down.shape == oref_down.shape == (nd, 3)
            np.testing.assert_allclose(down, oref_down, rtol=0, atol=1e-5)
            moved = float(np.abs(ref["points"] - s["raw"]).max())
            # ---- lasermap_fov_segment + Delete_Point_Boxes
            pos_lid = x_prop[0:3] + synth.quat_matrix(x_prop[3:7]) @ x_prop[11:14]
            deleted = lm.lasermap_fov_segment(pos_lid)
            oini, boxes = oracle_mod.fov_segment(pos_lid, omin, omax, oini, cube_len=124.0, det_range=40.0)
            np.testing.assert_array_equal(boxes, lm.last["fov_boxes"])
            assert deleted == om.delete_boxes(boxes)
            # ---- update_iterated_dyn_share_modified (reference control flow)
            nearest = {}
            lm.kf.update_iterated_dyn_share_modified(0.001, None, lm.ikdtree, nearest, 4, False)
            xg = lm.kf.get_x().to_array()
            op, oi = om.dump()
            T = oracle_mod.Tree(op)
            s_ref, P_ref, stats, idx_ref, sqd_ref, sel_ref = oracle_mod.ikf_update(
                T, down, x_prop, P_prop, maximum_iter=4, mode=0, reference_gain=0)
            assert np.abs(xg[0:3] - s_ref[0:3]).max() < 1e-4
            assert rot_err(xg[3:7], s_ref[3:7]) < 1e-5
            np.testing.assert_allclose(lm.kf.get_P(), P_ref, atol=1e-6 * np.abs(P_ref).max())
            # ---- map_incremental: the oracle's map driven by the oracle's own Nearest_Points
            counts_dev = lm.kf.map_incremental(lm.ikdtree, 0.5, True)
            ids_oracle = np.where(idx_ref >= 0, oi[np.maximum(idx_ref, 0)], -1).astype(np.int32)
            counts_orc = om.incremental(xg, down, ids_oracle, 0.5, True, 0.5)
            np.testing.assert_array_equal(counts_dev, counts_orc)
            if k % check_every == 0 or k == len(seq) - 1:
                assert_same_map(L, lm.ikdtree.h, om)
            report.append((k, nd, moved, float(np.abs(xg[0:3] - s["frame"].gt_pos).max()),
                           int(counts_dev[0] + counts_dev[1]), int(deleted)))
    finally:
        lm.kf.close()
        lm.ikdtree.close()
    return report


def test_scan_chain_sequence(L, oracle_mod):
    """11 scans (10 updates) of 20k raw points along the street, 200k map."""
    seq = make_sequence(20261015, 200_000, 11, 20_000, 0.6)
    rep = run_chain(L, oracle_mod, seq, None, 20_000)
    for k, nd, moved, err, added, deleted in rep:
        print(f"scan {k}: {nd} down, undistortion moved up to {moved:.3f} m, |x - gt| {err:.3f} m, "
              f"{added} map candidates, {deleted} deleted")
    assert len(rep) == 10
    assert max(r[2] for r in rep) > 0.1          # the undistortion moved points
    assert sum(r[4] for r in rep) > 0            # the map grew
    assert max(r[3] for r in rep) < 0.3          # and the scans stayed near the ground truth


def test_scan_chain_c2_size(L, oracle_mod):
    """Two scans at C2 size: 10M-point map, a 100k-point raw scan through the
    whole chain (the second scan is the checked one)."""
    seq = make_sequence(20261016, 10_000_000, 2, 100_000, 0.6)
    rep = run_chain(L, oracle_mod, seq, None, 100_000)
    assert len(rep) == 1 and rep[0][1] > 20_000
