"""The per-scan part of S-FAST_LIO's laserMapping main loop on the MI355X path.

Mirrors ``src/S-FAST_LIO/src/laserMapping.cpp:702-797`` from the point where a
downsampled scan (``feats_down_body``) and the propagated state exist:

  1. state_point = kf.get_x(); pos_lid = pos + rot * T_LI           (:727-730)
  2. lasermap_fov_segment(): move the local map box, Delete_Point_Boxes (:736, 309-365)
  3. skip scans with < 5 points                                      (:741-744)
  4. first scan: ikdtree.set_downsample_param; Build(feats_down_world) (:747-757)
  5. Nearest_Points.resize; kf.update_iterated_dyn_share_modified    (:771-774)
  6. map_incremental()                                               (:786, 382-433)

Every numeric step runs on the GPU through libslio (include/slio.h): the map
lives in HBM and is changed there (no re-upload), the IKF update is the
device-resident one.  This module only sequences the calls, like the ROS node.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import _lib as L
from .esekf import LASER_POINT_COV, Esekf, KdTreeMap, StateIkfom

INIT_TIME = 0.1          # laserMapping.cpp:28
DET_RANGE = 300.0        # laserMapping.cpp:39
NUM_MAX_ITERATIONS = 4   # laserMapping.cpp:604 (param default)


def quat_matrix(q: np.ndarray) -> np.ndarray:
    """Eigen Quaternion::toRotationMatrix (Sophus SO3::matrix), q = (w, x, y, z)."""
    w, x, y, z = (float(v) for v in q)
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1.0 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1.0 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1.0 - (txx + tyy)]])


def _mv(R: np.ndarray, v: np.ndarray) -> np.ndarray:
    # Eigen's 3x3 * 3-vector: ((r0*v0 + r1*v1) + r2*v2) per row, in double
    return (R[:, 0][:, None] * v[0] + R[:, 1][:, None] * v[1]) + R[:, 2][:, None] * v[2]


def point_body_to_world(x: StateIkfom, body: np.ndarray) -> np.ndarray:
    """pointBodyToWorld (laserMapping.cpp:276-287), rotation matrices, to float."""
    pb = np.asarray(body, dtype=np.float32)[:, :3].astype(np.float64).T
    a = _mv(quat_matrix(x.offset_R_L_I), pb) + np.asarray(x.offset_T_L_I, dtype=np.float64)[:, None]
    w = _mv(quat_matrix(x.rot), a) + np.asarray(x.pos, dtype=np.float64)[:, None]
    return w.T.astype(np.float32)


class _LazyNearest(dict):
    """Nearest_Points of the scan's last search pass, read from the device on
    first use: map_incremental runs on the device from the pass's neighbour
    positions, so the live loop never copies 100k x 5 ids to the host (the
    ids stay derivable until the handle's scan or map changes; valid until
    the next process())."""

    def __init__(self, kf):
        super().__init__()
        self._kf = kf
        self._loaded = False

    def _load(self):
        if not self._loaded:
            self._loaded = True
            super().update(self._kf.nearest_points())

    def __getitem__(self, k):
        self._load()
        return super().__getitem__(k)

    def __contains__(self, k):
        self._load()
        return super().__contains__(k)

    def __iter__(self):
        self._load()
        return super().__iter__()

    def __len__(self):
        self._load()
        return super().__len__()

    def get(self, k, default=None):
        self._load()
        return super().get(k, default)

    def keys(self):
        self._load()
        return super().keys()

    def items(self):
        self._load()
        return super().items()

    def values(self):
        self._load()
        return super().values()


class LaserMapping:
    """Per-scan driver of laserMapping with the map kept on the device."""

    def __init__(self, filter_size_map_min: float = 0.5, cube_len: float = 1000.0,
                 det_range: float = DET_RANGE, maximum_iter: int = NUM_MAX_ITERATIONS,
                 extrinsic_est: bool = False, device: int = 0, max_points: int = 100000,
                 grid_cell: float = 0.0):  # 0: the library's auto edge (slio_params.grid_cell)
        self.filter_size_map_min = float(filter_size_map_min)
        self.cube_len = float(cube_len)
        self.det_range = float(det_range)
        self.maximum_iter = int(maximum_iter)
        self.extrinsic_est = bool(extrinsic_est)
        self.ikdtree = KdTreeMap(device=device, grid_cell=grid_cell)
        self.kf = Esekf(device=device, max_points=max_points)
        self.built = False
        self.first_lidar_time = None
        self.local_min = np.zeros(3, np.float32)
        self.local_max = np.zeros(3, np.float32)
        self.local_init = C.c_int(0)
        self.Nearest_Points: dict = {}
        self.last = {}

    def lasermap_fov_segment(self, pos_lid: np.ndarray) -> int:
        """laserMapping.cpp:309-365; returns kdtree_delete_counter."""
        boxes = np.zeros(18, np.float32)
        nb = C.c_int(0)
        pos = np.ascontiguousarray(pos_lid, dtype=np.float64)
        L.check(L.load().slio_fov_segment(L.dptr(pos), L.fptr(self.local_min), L.fptr(self.local_max),
                                          C.byref(self.local_init), self.cube_len, self.det_range,
                                          L.fptr(boxes), C.byref(nb)), "lasermap_fov_segment")
        self.last["fov_boxes"] = boxes[:6 * nb.value].reshape(-1, 6).copy()
        if nb.value == 0 or not self.built:
            return 0
        return self.ikdtree.Delete_Point_Boxes(self.last["fov_boxes"])

    def process(self, feats_down_body: np.ndarray, lidar_beg_time: float) -> bool:
        """One scan; the filter's state/covariance (kf.get_x / get_P) must hold
        the propagated prior.  Returns False when the scan was skipped or only
        built the map (as the reference's `continue`)."""
        if self.first_lidar_time is None:
            self.first_lidar_time = float(lidar_beg_time)
        x = self.kf.get_x()
        pos_lid = np.asarray(x.pos, dtype=np.float64) + _mv(
            quat_matrix(x.rot), np.asarray(x.offset_T_L_I, dtype=np.float64)[:, None])[:, 0]
        flg_ekf_inited = (float(lidar_beg_time) - self.first_lidar_time) >= INIT_TIME
        t0 = time.perf_counter()
        self.last["deleted"] = self.lasermap_fov_segment(pos_lid)
        t1 = time.perf_counter()
        body = np.ascontiguousarray(np.asarray(feats_down_body, dtype=np.float32)[:, :3])
        if body.shape[0] < 5:
            return False
        if not self.built:
            self.ikdtree.set_downsample_param(self.filter_size_map_min)
            self.ikdtree.Build(point_body_to_world(x, body))
            self.built = True
            return False
        self.kf.update_iterated_dyn_share_modified(LASER_POINT_COV, body, self.ikdtree, None,
                                                   self.maximum_iter, self.extrinsic_est)
        self.Nearest_Points = _LazyNearest(self.kf)
        t2 = time.perf_counter()
        self.last["map_incremental"] = self.kf.map_incremental(self.ikdtree, self.filter_size_map_min,
                                                               flg_ekf_inited)
        t3 = time.perf_counter()
        # host wall clock of the three steps (ms): fov segment + deletions,
        # scan upload + IKF update, map_incremental
        self.last["t_ms"] = (1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2))
        return True
