"""ImuProcess::UndistortPcl on the MI355X path.

Mirrors ``src/S-FAST_LIO/src/IMU_Processing.hpp`` (class ImuProcess,
:253-402): the forward propagation of the filter over the scan's IMU samples
(esekf::predict, esekfom.hpp:82-95) is a short sequential 24-D recursion and
runs on the host in C++ (slio_imu_forward); the per-point back-propagation to
the scan end runs on the device (slio_undistort / the device pipeline
slio_scan_upload_undistort_voxel, which hands the undistorted, downsampled
scan to the IKF without leaving HBM).  IMU initialisation (IMU_init, the
first scans' mean acceleration / gyro bias) is the caller's: mean_acc and the
noise covariances are plain members here.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .esekf import Esekf, StateIkfom


@dataclass
class MeasureGroup:
    """common_lib.h MeasureGroup: one scan with its IMU samples."""
    lidar_beg_time: float
    lidar_end_time: float
    points: np.ndarray             # (n, 3) float32, LiDAR frame
    t_ms: np.ndarray               # (n,) float32, per-point offset from lidar_beg_time (curvature)
    imu: np.ndarray                # (k, 7): stamp, acc xyz, gyr xyz


@dataclass
class ImuProcess:
    mean_acc: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, -1.0]))
    cov_gyr: np.ndarray = field(default_factory=lambda: np.full(3, 0.1))
    cov_acc: np.ndarray = field(default_factory=lambda: np.full(3, 0.1))
    cov_bias_gyr: np.ndarray = field(default_factory=lambda: np.full(3, 0.0001))
    cov_bias_acc: np.ndarray = field(default_factory=lambda: np.full(3, 0.0001))
    last_imu_: np.ndarray | None = None
    acc_s_last: np.ndarray = field(default_factory=lambda: np.zeros(3))
    angvel_last: np.ndarray = field(default_factory=lambda: np.zeros(3))
    last_lidar_end_time_: float = 0.0
    IMUpose: list = field(default_factory=list)

    def _forward(self, meas: MeasureGroup, kf: Esekf):
        v_imu = np.asarray(meas.imu, dtype=np.float64).reshape(-1, 7)
        if self.last_imu_ is not None:
            v_imu = np.concatenate([self.last_imu_[None], v_imu])   # v_imu.push_front(last_imu_)
        samples = (L.SlioImuSample * v_imu.shape[0])()
        for k, r in enumerate(v_imu):
            samples[k].t = r[0]
            samples[k].acc[:] = list(r[1:4])
            samples[k].gyr[:] = list(r[4:7])
        poses = (L.SlioImuPose * v_imu.shape[0])()
        npose = C.c_int()
        lle = C.c_double(self.last_lidar_end_time_)
        xs = kf.get_x().to_c()
        P = np.ascontiguousarray(kf.get_P(), dtype=np.float64).copy()
        asl = np.ascontiguousarray(self.acc_s_last, dtype=np.float64).copy()
        avl = np.ascontiguousarray(self.angvel_last, dtype=np.float64).copy()
        cov = [np.ascontiguousarray(c, dtype=np.float64) for c in
               (self.cov_gyr, self.cov_acc, self.cov_bias_gyr, self.cov_bias_acc)]
        L.check(L.load().slio_imu_forward(samples, v_imu.shape[0], meas.lidar_beg_time, meas.lidar_end_time,
                                          C.byref(lle), float(np.linalg.norm(self.mean_acc)),
                                          *(L.dptr(c) for c in cov), L.dptr(asl), L.dptr(avl), C.byref(xs),
                                          L.dptr(P), poses, v_imu.shape[0], C.byref(npose)), "UndistortPcl")
        kf.change_x(StateIkfom.from_c(xs))
        kf.change_P(P)
        self.acc_s_last, self.angvel_last = asl, avl
        self.last_lidar_end_time_ = lle.value
        self.last_imu_ = np.asarray(meas.imu, dtype=np.float64).reshape(-1, 7)[-1].copy()
        self.IMUpose = poses[:npose.value]
        return poses, npose.value, xs

    def UndistortPcl(self, meas: MeasureGroup, kf: Esekf) -> tuple[np.ndarray, np.ndarray]:
        """IMU_Processing.hpp:253-402: predicts kf over the scan and returns
        feats_undistort (points in time order, their times in ms)."""
        poses, npose, xs = self._forward(meas, kf)
        pts = np.ascontiguousarray(np.asarray(meas.points, dtype=np.float32)[:, :3])
        n = pts.shape[0]
        x, y, z = (np.ascontiguousarray(pts[:, k]) for k in range(3))
        t = np.ascontiguousarray(meas.t_ms, dtype=np.float32)
        ox, oy, oz, ot = (np.zeros(n, np.float32) for _ in range(4))
        L.check(L.load().slio_undistort(kf.h, L.fptr(x), L.fptr(y), L.fptr(z), L.fptr(t), n, poses, npose,
                                        C.byref(xs), L.fptr(ox), L.fptr(oy), L.fptr(oz), L.fptr(ot)),
                "UndistortPcl")
        return np.stack([ox, oy, oz], 1), ot

    def undistort_downsample(self, meas: MeasureGroup, kf: Esekf, filter_size_surf: float) -> int:
        """UndistortPcl + downSizeFilterSurf without leaving the device: the
        result is kf's feats_down_body (pass None as the scan to the update).
        Returns feats_down_size."""
        poses, npose, xs = self._forward(meas, kf)
        pts = np.ascontiguousarray(np.asarray(meas.points, dtype=np.float32)[:, :3])
        x, y, z = (np.ascontiguousarray(pts[:, k]) for k in range(3))
        t = np.ascontiguousarray(meas.t_ms, dtype=np.float32)
        nd = C.c_int64()
        L.check(L.load().slio_scan_upload_undistort_voxel(kf.h, L.fptr(x), L.fptr(y), L.fptr(z), L.fptr(t),
                                                          pts.shape[0], poses, npose, C.byref(xs),
                                                          float(filter_size_surf), C.byref(nd)),
                "undistort_downsample")
        kf._scan_ref = None
        kf._n_scan = int(nd.value)
        return kf._n_scan
