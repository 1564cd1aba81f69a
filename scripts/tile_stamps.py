"""Per-block phase timing of the tiled search pass (diagnostic build with
-DSLIO_ABL_STAMP, SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_STAMP.so): start,
queries formed, first tile staged, first batch searched, kNN done, fit
done, end (s_memrealtime, 100 MHz)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

lib = L.load(os.environ["SLIO_LIB"])
lib.slio_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
if os.environ.get("ORDER", "voxel") == "voxel":
    fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
st = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI])
pose = L.SlioPose()
pose.pos[:] = list(st[0:3]); pose.rot[:] = list(st[3:7])
pose.rli[:] = list(st[7:11]); pose.tli[:] = list(st[11:14])
p = L.SlioParams(); lib.slio_params_default(C.byref(p)); p.grid_cell = float(os.environ.get("CELL", "1.25"))
h = C.c_void_p(); L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
HTH = np.zeros(78); HTh = np.zeros(12); m = C.c_int64()
for _ in range(5):
    L.check(lib.slio_iterate(h, C.byref(pose), 1, 0, L.dptr(HTH), L.dptr(HTh), C.byref(m)), "it")
nb = (fr.body.shape[0] + 127) // 128
buf = (C.c_ulonglong * (8 * nb))()
assert lib.slio_debug_stamps(buf, nb) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
t0 = a[:, 0].min()
us = (a - t0) / 100.0
print(f"blocks={nb}: kernel span {us[:, 3].max():.1f}us; start spread {us[:, 0].max():.1f}us")
for name, (i, j) in (("queries", (0, 4)), ("hash", (4, 7)), ("stage1", (4, 5)), ("batch1", (5, 6)), ("knn-all", (4, 1)),
                     ("fit", (1, 2)), ("prod", (2, 3)), ("total", (0, 3))):
    v = us[:, j] - us[:, i]
    print(f"  {name:8s} mean {v.mean():7.2f} p50 {np.median(v):7.2f} p90 {np.quantile(v, .9):7.2f} max {v.max():7.2f} us")
lib.slio_destroy(h)
