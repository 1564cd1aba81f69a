"""LIO-SAM scan-to-map optimisation on the MI355X path.

Mirrors ``src/LIO-SAM/src/mapOptmization.cpp`` scan2MapOptimization
(:1706-1740) and the functions it calls: cornerOptimization (:1303-1432),
surfOptimization (:1438-1515), combineOptimizationCoeffs (:1517-1543) and
LMOptimization (:1552-1700).  The per-point work (pointAssociateToMap, exact
5-NN in the corner / surf local maps, line and plane fits, the LM rows and
the normal equations) runs on the device through libslio; the 6x6 step is
host C++ (slio_s2m_lm_step).  transformUpdate's IMU blending (:1742-1781)
and the keyframe / factor-graph back end are out of scope (SURVEY.md §8f-4
names the scan-to-map core).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

EDGE_FEATURE_MIN_VALID_NUM = 10    # params.yaml edgeFeatureMinValidNum
SURF_FEATURE_MIN_VALID_NUM = 100   # params.yaml surfFeatureMinValidNum


def _handle(max_points: int, grid_cell: float, device: int = 0):
    lib = L.load()
    p = L.SlioParams()
    L.check(lib.slio_params_default(C.byref(p)), "params")
    p.device, p.max_points, p.grid_cell = device, max_points, grid_cell
    h = C.c_void_p()
    L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
    return h


def _upload(lib, fn, h, pts):
    pts = np.ascontiguousarray(np.asarray(pts, dtype=np.float32).reshape(-1, 3))
    x, y, z = (np.ascontiguousarray(pts[:, k]) for k in range(3))
    L.check(fn(h, L.fptr(x), L.fptr(y), L.fptr(z), pts.shape[0]), fn.__name__)
    return pts.shape[0]


class ScanToMap:
    """kdtreeCornerFromMap / kdtreeSurfFromMap and the scan-to-map solve."""

    def __init__(self, max_points: int = 200000, grid_cell: float = 1.0, device: int = 0):
        self.lib = L.load()
        self.hc = _handle(max_points, grid_cell, device)
        self.hs = _handle(max_points, grid_cell, device)
        self.n_corner = self.n_surf = 0
        self.isDegenerate = C.c_int(0)
        self.matP = np.zeros(36, np.float32)
        self.iterations = 0

    def close(self):
        for h in (self.hc, self.hs):
            if h:
                self.lib.slio_destroy(h)
        self.hc = self.hs = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_maps(self, corner_from_map_ds: np.ndarray, surf_from_map_ds: np.ndarray) -> None:
        """kdtree{Corner,Surf}FromMap->setInputCloud (:1716-1717)."""
        _upload(self.lib, self.lib.slio_map_upload, self.hc, corner_from_map_ds)
        _upload(self.lib, self.lib.slio_map_upload, self.hs, surf_from_map_ds)

    def set_scan(self, corner_last_ds: np.ndarray, surf_last_ds: np.ndarray) -> None:
        """laserCloud{Corner,Surf}LastDS of the current frame."""
        self.n_corner = _upload(self.lib, self.lib.slio_scan_upload, self.hc, corner_last_ds)
        self.n_surf = _upload(self.lib, self.lib.slio_scan_upload, self.hs, surf_last_ds)

    def corner_optimization(self, transform: np.ndarray, count: bool = True) -> int:
        """:1303-1432; count: return the selected points (a device -> host
        copy and a wait; the LM loop takes the count from the normal
        equations instead)."""
        k = C.c_int64()
        L.check(self.lib.slio_s2m_coeffs(self.hc, 0, L.fptr(transform), C.byref(k) if count else None),
                "cornerOptimization")
        return k.value

    def surf_optimization(self, transform: np.ndarray, count: bool = True) -> int:
        """:1438-1515 (see corner_optimization)."""
        k = C.c_int64()
        L.check(self.lib.slio_s2m_coeffs(self.hs, 1, L.fptr(transform), C.byref(k) if count else None),
                "surfOptimization")
        return k.value

    def normal_equations(self, transform: np.ndarray):
        AtA = np.zeros(36, np.float32)
        AtB = np.zeros(6, np.float32)
        n = C.c_int64()
        L.check(self.lib.slio_s2m_normal_equations(self.hc, self.hs, L.fptr(transform), L.fptr(AtA), L.fptr(AtB),
                                                   C.byref(n)), "normal_equations")
        return AtA, AtB, n.value

    def LMOptimization(self, transform: np.ndarray, iter_count: int) -> bool:
        AtA, AtB, nsel = self.normal_equations(transform)
        conv = C.c_int(0)
        rc = self.lib.slio_s2m_lm_step(L.fptr(AtA), L.fptr(AtB), nsel, iter_count, L.fptr(transform),
                                       C.byref(self.isDegenerate), L.fptr(self.matP), C.byref(conv))
        if rc < 0:
            L.check(rc, "LMOptimization")
        return bool(conv.value)

    def scan2MapOptimization(self, transformTobeMapped: np.ndarray) -> np.ndarray:
        """:1706-1740 -- returns the optimised transformTobeMapped (roll,
        pitch, yaw, x, y, z); unchanged when the frame has too few features."""
        tf = np.ascontiguousarray(transformTobeMapped, dtype=np.float32).copy()
        self.iterations = 0
        if not (self.n_corner > EDGE_FEATURE_MIN_VALID_NUM and self.n_surf > SURF_FEATURE_MIN_VALID_NUM):
            return tf
        for it in range(30):
            self.corner_optimization(tf, count=False)
            self.surf_optimization(tf, count=False)
            self.iterations = it + 1
            if self.LMOptimization(tf, it):
                break
        return tf
