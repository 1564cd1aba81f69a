"""Run the kNN golden case against a given library build (SLIO_LIB), e.g. the
SLIO_BOUNDS_CHECK diagnostic build; prints mismatch counts."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L  # noqa: E402

lib = L.load(os.environ.get("SLIO_LIB", L.LIB_PATH))
z = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "knn_golden.npz"))
p = L.SlioParams()
lib.slio_params_default(C.byref(p))
p.max_points, p.grid_cell, p.far_query_margin = 100000, float(os.environ.get("CELL", "0.75")), 0.0
h = C.c_void_p()
L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
mp = np.ascontiguousarray(z["map"], np.float32)
x, y, zz = (np.ascontiguousarray(mp[:, k]) for k in range(3))
L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(zz), mp.shape[0]), "map")
q = np.ascontiguousarray(z["query"], np.float32)
qx, qy, qz = (np.ascontiguousarray(q[:, k]) for k in range(3))
L.check(lib.slio_scan_upload(h, L.fptr(qx), L.fptr(qy), L.fptr(qz), q.shape[0]), "scan")
pose = L.SlioPose()
pose.rot[:] = [1, 0, 0, 0]
pose.rli[:] = [1, 0, 0, 0]
HTH = np.zeros(78); HTh = np.zeros(12); m = C.c_int64()
L.check(lib.slio_iterate(h, C.byref(pose), 1, 0, L.dptr(HTH), L.dptr(HTh), C.byref(m)), "iterate")
n = q.shape[0]
idx = np.zeros((n, 5), np.int32); sqd = np.zeros((n, 5), np.float32); sel = np.zeros(n, np.uint8)
L.check(lib.slio_get_neighbors(h, L.iptr(idx), L.fptr(sqd), L.u8ptr(sel)), "neighbors")
print("idx mismatches", int((idx != z["idx"]).any(1).sum()), "sqd mismatches",
      int((sqd != z["sqd"]).any(1).sum()), "of", n, flush=True)
lib.slio_destroy(h)
