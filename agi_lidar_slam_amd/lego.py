"""Host side of the LeGO-LOAM front-end, mirroring
ImageProjection (LeGO-LOAM/src/imageProjection.cpp) and the front half of
FeatureAssociation (featureAssociation.cpp: adjustDistortion,
calculateSmoothness, markOccludedPoints, extractFeatures).

The IMU ring buffer that adjustDistortion reads is host state filled message
by message (imuHandler + AccumulateIMUShiftAndRotation, :430-588); `LegoImu`
restates it.  The device side lives behind include/slio_frontend.h
(slio_lego_*).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass

import numpy as np

from . import _lib as L

IMU_QUE_LEN = 200  # imuQueLength (utility.h:42)


@dataclass
class LegoParams:
    """LeGO-LOAM/include/utility.h:20-49 (VLP-16) and the less-flat VoxelGrid
    leaf of featureAssociation.cpp:222."""
    N_SCAN: int = 16
    Horizon_SCAN: int = 1800
    ang_res_x: float = 0.2
    ang_res_y: float = 2.0
    ang_bottom: float = 15.0 + 0.1
    groundScanInd: int = 7
    sensorMountAngle: float = 0.0
    segmentTheta: float = 1.0472
    segmentValidPointNum: int = 5
    segmentValidLineNum: int = 3
    edgeThreshold: float = 0.1
    surfThreshold: float = 0.1
    leafSize: float = 0.2
    scanPeriod: float = 0.1

    def to_c(self, device: int = 0, max_points: int = 0) -> L.SlioLegoParams:
        p = L.SlioLegoParams()
        L.load().slio_lego_params_default(C.byref(p))
        p.device, p.max_points = device, max_points
        p.n_scan, p.horizon_scan, p.ground_scan_ind = self.N_SCAN, self.Horizon_SCAN, self.groundScanInd
        p.segment_valid_point_num = self.segmentValidPointNum
        p.segment_valid_line_num = self.segmentValidLineNum
        p.ang_res_x, p.ang_res_y, p.ang_bottom = self.ang_res_x, self.ang_res_y, self.ang_bottom
        p.sensor_mount_angle, p.segment_theta = self.sensorMountAngle, self.segmentTheta
        p.edge_threshold, p.surf_threshold = self.edgeThreshold, self.surfThreshold
        p.leaf_size, p.scan_period = self.leafSize, self.scanPeriod
        return p


class LegoImu:
    """FeatureAssociation's IMU ring buffer (featureAssociation.cpp:109-132):
    imuHandler (:559-587) + AccumulateIMUShiftAndRotation (:430-557), and the
    pointers / angular rotation adjustDistortion carries between scans."""

    def __init__(self, que_len: int = IMU_QUE_LEN, scan_period: float = 0.1):
        f = lambda: np.zeros(que_len, np.float32)  # noqa: E731
        self.Q = que_len
        self.scan_period = scan_period
        self.time = np.zeros(que_len, np.float64)
        self.roll, self.pitch, self.yaw = f(), f(), f()
        self.acc_x, self.acc_y, self.acc_z = f(), f(), f()
        self.velo_x, self.velo_y, self.velo_z = f(), f(), f()
        self.shift_x, self.shift_y, self.shift_z = f(), f(), f()
        self.angvel_x, self.angvel_y, self.angvel_z = f(), f(), f()
        self.ang_x, self.ang_y, self.ang_z = f(), f(), f()
        self.pointer_last = -1
        self.pointer_last_iteration = 0
        self.ang_last = np.zeros(3, np.float32)

    def imuHandler(self, stamp: float, roll: float, pitch: float, yaw: float, acc, gyro):
        f32 = np.float32
        ax = f32(acc[1] - math.sin(roll) * math.cos(pitch) * 9.81)
        ay = f32(acc[2] - math.cos(roll) * math.cos(pitch) * 9.81)
        az = f32(acc[0] + math.sin(pitch) * 9.81)
        p = self.pointer_last = (self.pointer_last + 1) % self.Q
        self.time[p] = stamp
        self.roll[p], self.pitch[p], self.yaw[p] = roll, pitch, yaw
        self.acc_x[p], self.acc_y[p], self.acc_z[p] = ax, ay, az
        self.angvel_x[p], self.angvel_y[p], self.angvel_z[p] = gyro
        self._accumulate()

    def _accumulate(self):
        f32 = np.float32
        p = self.pointer_last
        r, pi, yw = f32(self.roll[p]), f32(self.pitch[p]), f32(self.yaw[p])
        ax, ay, az = self.acc_x[p], self.acc_y[p], self.acc_z[p]
        c, s = f32(math.cos(r)), f32(math.sin(r))
        x1, y1, z1 = f32(c * ax - s * ay), f32(s * ax + c * ay), az
        c, s = f32(math.cos(pi)), f32(math.sin(pi))
        x2, y2, z2 = x1, f32(c * y1 - s * z1), f32(s * y1 + c * z1)
        c, s = f32(math.cos(yw)), f32(math.sin(yw))
        ax, ay, az = f32(c * x2 + s * z2), y2, f32(-s * x2 + c * z2)
        b = (p + self.Q - 1) % self.Q
        dt = self.time[p] - self.time[b]
        if dt < self.scan_period:
            for sh, ve, a in ((self.shift_x, self.velo_x, ax), (self.shift_y, self.velo_y, ay),
                              (self.shift_z, self.velo_z, az)):
                sh[p] = f32(sh[b] + ve[b] * dt + a * dt * dt / 2)
                ve[p] = f32(ve[b] + a * dt)
            for an, av in ((self.ang_x, self.angvel_x), (self.ang_y, self.angvel_y),
                           (self.ang_z, self.angvel_z)):
                an[p] = f32(an[b] + av[b] * dt)

    def feed(self, imu: dict, until: float):
        """imuHandler for every message of a synth stream up to `until`."""
        for k in range(imu["time"].size):
            if imu["time"][k] > until:
                break
            self.imuHandler(float(imu["time"][k]), float(imu["roll"][k]), float(imu["pitch"][k]),
                            float(imu["yaw"][k]), imu["acc"][k], imu["gyro"][k])


class LegoFrontEnd:
    """ImageProjection::cloudHandler + the front half of
    FeatureAssociation::runFeatureAssociation (adjustDistortion ..
    extractFeatures) as one device pipeline (slio_lego_run): the range image,
    segmentation and cloud_info never leave HBM.  No CPU fallback: without
    libslio.so the constructor raises."""

    def __init__(self, params: LegoParams | None = None, device: int = 0, max_points: int = 0):
        self.params = params or LegoParams()
        self.lib = L.load()
        self.h = C.c_void_p()
        self._p = self.params.to_c(device, max_points)
        L.check(self.lib.slio_lego_create(C.byref(self.h), C.byref(self._p)), "slio_lego_create")
        self.counts = L.SlioLegoCounts()

    def close(self):
        if self.h:
            self.lib.slio_lego_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_imu(self, imu: LegoImu | None, time_scan_cur: float = 0.0):
        """The IMU state adjustDistortion reads (None: imuPointerLast = -1)."""
        if imu is None:
            L.check(self.lib.slio_lego_set_imu(self.h, None), "set_imu")
            return
        keep = [np.ascontiguousarray(imu.time, np.float64)]
        arrs = []
        for n in ("roll", "pitch", "yaw", "velo_x", "velo_y", "velo_z", "shift_x", "shift_y",
                  "shift_z", "ang_x", "ang_y", "ang_z"):
            a = np.ascontiguousarray(getattr(imu, n), np.float32)
            keep.append(a)
            arrs.append(L.fptr(a))
        s = L.SlioLegoImu(L.dptr(keep[0]), *arrs, imu.pointer_last, imu.pointer_last_iteration,
                          imu.Q, float(time_scan_cur), (C.c_float * 3)(*imu.ang_last))
        L.check(self.lib.slio_lego_set_imu(self.h, C.byref(s)), "set_imu")

    def upload(self, x, y, z):
        f = [np.ascontiguousarray(v, dtype=np.float32) for v in (x, y, z)]
        self._keep = f
        L.check(self.lib.slio_lego_upload(self.h, *(L.fptr(v) for v in f), len(f[0])), "upload")

    def run(self) -> L.SlioLegoCounts:
        L.check(self.lib.slio_lego_run(self.h, C.byref(self.counts)), "slio_lego_run")
        return self.counts

    def cloudHandler(self, x, y, z, imu: LegoImu | None = None, time_scan_cur: float = 0.0):
        """One sweep through imageProjection + featureAssociation's front half;
        carries the IMU pointers / angular rotation into `imu` as the
        reference does between scans."""
        self.set_imu(imu, time_scan_cur)
        self.upload(x, y, z)
        self.run()
        f = self.features()
        if imu is not None:
            imu.pointer_last_iteration = f["imu_out"]["pointer_last_iteration"]
            imu.ang_last = np.asarray(f["imu_out"]["ang_last"], np.float32)
        return f

    # --------------------------------------------------------------- outputs
    def image(self) -> dict:
        N, H = self.params.N_SCAN, self.params.Horizon_SCAN
        rm = np.empty((N, H), np.float32)
        own = np.empty((N, H), np.int32)
        gr = np.empty((N, H), np.int8)
        lb = np.empty((N, H), np.int32)
        L.check(self.lib.slio_lego_get_image(self.h, L.fptr(rm), L.iptr(own),
                                             gr.ctypes.data_as(C.POINTER(C.c_int8)), L.iptr(lb)),
                "image")
        return dict(range_mat=rm, cell_point=own, ground=gr, label=lb)

    def seg_info(self) -> dict:
        c, R = self.counts, self.params.N_SCAN
        n, no = c.n_segmented, c.n_outlier
        st, en = np.empty(R, np.int32), np.empty(R, np.int32)
        gf, ci, sr = np.empty(n, np.uint8), np.empty(n, np.int32), np.empty(n, np.float32)
        sx, ox = np.empty((n, 4), np.float32), np.empty((no, 4), np.float32)
        L.check(self.lib.slio_lego_get_seg_info(self.h, L.iptr(st), L.iptr(en), L.u8ptr(gf),
                                                L.iptr(ci), L.fptr(sr), L.fptr(sx), L.fptr(ox)),
                "seg_info")
        return dict(orientation=np.array(c.orientation, np.float32), startRingIndex=st,
                    endRingIndex=en, segmentedCloudGroundFlag=gf, segmentedCloudColInd=ci,
                    segmentedCloudRange=sr, segmented_cloud=sx, outlier_cloud=ox)

    def features(self) -> dict:
        c = self.counts
        n = c.n_segmented
        dk = np.empty((n, 4), np.float32)
        cv, pk, lb = np.empty(n, np.float32), np.empty(n, np.uint8), np.empty(n, np.int32)
        io = L.SlioLegoImuOut()
        L.check(self.lib.slio_lego_get_features(self.h, L.fptr(dk), L.fptr(cv), L.u8ptr(pk),
                                                L.iptr(lb), C.byref(io)), "features")
        out = [np.empty((k, 4), np.float32) for k in (c.n_sharp, c.n_less_sharp, c.n_flat,
                                                       c.n_less_flat)]
        L.check(self.lib.slio_lego_get_clouds(self.h, *(L.fptr(v) for v in out)), "clouds")
        return dict(deskewed=dk, cloudCurvature=cv, cloudNeighborPicked=pk, cloudLabel=lb,
                    cornerPointsSharp=out[0], cornerPointsLessSharp=out[1], surfPointsFlat=out[2],
                    surfPointsLessFlat=out[3],
                    imu_out=dict(rpy_start=np.array(io.rpy_start), rpy_cur=np.array(io.rpy_cur),
                                 velo_from_start=np.array(io.velo_from_start),
                                 angular_from_start=np.array(io.angular_from_start),
                                 ang_last=np.array(io.ang_last),
                                 pointer_last_iteration=io.pointer_last_iteration))
