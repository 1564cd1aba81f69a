"""Host side of the LIO-SAM front-end, mirroring
ImageProjection / FeatureExtraction (LIO-SAM/src/imageProjection.cpp,
featureExtraction.cpp) over the C-ABI of include/slio_frontend.h.

ImageProjection.cloudHandler (imageProjection.cpp:193-212) keeps the host
parts -- IMU queue bookkeeping (imuDeskewInfo :345-392, restated in
`imu_deskew_table`) -- and runs projectPointCloud / cloudExtraction on the
device; FeatureExtraction.laserCloudInfoHandler (featureExtraction.cpp:88-100)
runs calculateSmoothness / markOccludedPoints / extractFeatures on the device.
Both stages are one device pipeline (slio_lio_run), so the cloud_info never
leaves HBM between them.  There is no CPU fallback: without libslio.so the
constructor raises.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L


@dataclass
class LioSamParams:
    """params.yaml:26-63 (defaults: VLP-16)."""
    N_SCAN: int = 16
    Horizon_SCAN: int = 1800
    downsampleRate: int = 1
    lidarMinRange: float = 1.0
    lidarMaxRange: float = 1000.0
    edgeThreshold: float = 1.0
    surfThreshold: float = 0.1
    odometrySurfLeafSize: float = 0.4

    def to_c(self, device: int = 0, max_points: int = 0) -> L.SlioLioParams:
        p = L.SlioLioParams()
        L.load().slio_lio_params_default(C.byref(p))
        p.device, p.max_points = device, max_points
        p.n_scan, p.horizon_scan, p.downsample_rate = self.N_SCAN, self.Horizon_SCAN, self.downsampleRate
        p.lidar_min_range, p.lidar_max_range = self.lidarMinRange, self.lidarMaxRange
        p.edge_threshold, p.surf_threshold = self.edgeThreshold, self.surfThreshold
        p.surf_leaf_size = self.odometrySurfLeafSize
        return p


def imu_deskew_table(stamps: np.ndarray, gyro: np.ndarray, time_scan_cur: float,
                     time_scan_end: float):
    """imuDeskewInfo (imageProjection.cpp:345-392): integrate the IMU angular
    velocity over [timeScanCur - 0.01, timeScanEnd + 0.01].  Returns
    (imuTime, imuRotX, imuRotY, imuRotZ) of length imuPointerCur + 1 and
    imuAvailable."""
    stamps = np.asarray(stamps, dtype=np.float64)
    keep = np.nonzero(stamps >= time_scan_cur - 0.01)[0]  # imuQueue.pop_front()
    if keep.size == 0:
        return (np.zeros(0),) * 4 + (False,)
    t, rx, ry, rz = [], [], [], []
    for i in range(keep[0], stamps.size):
        cur = float(stamps[i])
        if cur > time_scan_end + 0.01:
            break
        if not t:
            t.append(cur)
            rx.append(0.0)
            ry.append(0.0)
            rz.append(0.0)
            continue
        dt = cur - t[-1]
        rx.append(rx[-1] + float(gyro[i, 0]) * dt)
        ry.append(ry[-1] + float(gyro[i, 1]) * dt)
        rz.append(rz[-1] + float(gyro[i, 2]) * dt)
        t.append(cur)
    n = len(t)
    return (np.array(t), np.array(rx), np.array(ry), np.array(rz), n - 1 > 0)


class LioSamFrontEnd:
    """ImageProjection + FeatureExtraction on one MI355X handle."""

    def __init__(self, params: LioSamParams | None = None, device: int = 0, max_points: int = 0):
        self.params = params or LioSamParams()
        self.lib = L.load()
        self.h = C.c_void_p()
        self._p = self.params.to_c(device, max_points)
        L.check(self.lib.slio_lio_create(C.byref(self.h), C.byref(self._p)), "slio_lio_create")
        self.counts = L.SlioLioCounts()

    def close(self):
        if self.h:
            self.lib.slio_lio_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --------------------------------------------------------------- stages
    def set_deskew(self, imu_time, rot_x, rot_y, rot_z, time_scan_cur: float, enabled: bool):
        a = [np.ascontiguousarray(v, dtype=np.float64) for v in (imu_time, rot_x, rot_y, rot_z)]
        L.check(self.lib.slio_lio_set_deskew(self.h, *(L.dptr(v) for v in a), len(a[0]),
                                             float(time_scan_cur), int(bool(enabled))), "deskew")

    def upload(self, x, y, z, intensity, ring, time):
        f = [np.ascontiguousarray(v, dtype=np.float32) for v in (x, y, z, intensity)]
        rg = np.ascontiguousarray(ring, dtype=np.uint16)
        tm = np.ascontiguousarray(time, dtype=np.float32)
        self._keep = (f, rg, tm)
        L.check(self.lib.slio_lio_upload(self.h, *(L.fptr(v) for v in f), L.u16ptr(rg), L.fptr(tm),
                                         len(rg)), "upload")

    def run(self) -> L.SlioLioCounts:
        L.check(self.lib.slio_lio_run(self.h, C.byref(self.counts)), "slio_lio_run")
        return self.counts

    def cloudHandler(self, scan: dict) -> dict:
        """imageProjection.cpp:193-212 for a synth.make_ouster_scan-style dict,
        followed by the feature stage; returns cloud_info."""
        t, rx, ry, rz, ok = imu_deskew_table(scan["imu_stamps"], scan["imu_gyro"],
                                             scan["time_scan_cur"], scan["time_scan_end"])
        self.set_deskew(t, rx, ry, rz, scan["time_scan_cur"], ok)
        self.upload(scan["x"], scan["y"], scan["z"], scan["intensity"], scan["ring"], scan["time"])
        self.run()
        return self.cloud_info()

    # --------------------------------------------------------------- outputs
    def range_image(self):
        p = self.params
        rm = np.empty((p.N_SCAN, p.Horizon_SCAN), np.float32)
        own = np.empty((p.N_SCAN, p.Horizon_SCAN), np.int32)
        L.check(self.lib.slio_lio_get_range_image(self.h, L.fptr(rm), L.iptr(own)), "range_image")
        return rm, own

    def cloud_info(self) -> dict:
        n, R = self.counts.n_extracted, self.params.N_SCAN
        st, en = np.empty(R, np.int32), np.empty(R, np.int32)
        ci, pr = np.empty(n, np.int32), np.empty(n, np.float32)
        xyzi = np.empty((n, 4), np.float32)
        L.check(self.lib.slio_lio_get_cloud_info(self.h, L.iptr(st), L.iptr(en), L.iptr(ci),
                                                 L.fptr(pr), L.fptr(xyzi)), "cloud_info")
        return dict(startRingIndex=st, endRingIndex=en, pointColInd=ci, pointRange=pr,
                    cloud_deskewed=xyzi)

    def features(self) -> dict:
        n = self.counts.n_extracted
        cv, pk, lb = np.empty(n, np.float32), np.empty(n, np.uint8), np.empty(n, np.int32)
        L.check(self.lib.slio_lio_get_features(self.h, L.fptr(cv), L.u8ptr(pk), L.iptr(lb)),
                "features")
        co = np.empty((self.counts.n_corner, 4), np.float32)
        su = np.empty((self.counts.n_surface, 4), np.float32)
        L.check(self.lib.slio_lio_get_clouds(self.h, L.fptr(co), L.fptr(su)), "clouds")
        return dict(cloudCurvature=cv, cloudNeighborPicked=pk, cloudLabel=lb, cloud_corner=co,
                    cloud_surface=su)
