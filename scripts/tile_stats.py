"""Tile staging statistics of the C2 search pass (diagnostic build with
-DSLIO_TILE_STATS; SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_tstat.so).
Env: CELL, ORDER (voxel|capture)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

lib = L.load(os.environ["SLIO_LIB"])
lib.slio_dbg_tile_stats.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
if os.environ.get("ORDER", "voxel") == "voxel":
    fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
st = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI])
pose = L.SlioPose()
pose.pos[:] = list(st[0:3]); pose.rot[:] = list(st[3:7])
pose.rli[:] = list(st[7:11]); pose.tli[:] = list(st[11:14])
p = L.SlioParams()
lib.slio_params_default(C.byref(p))
p.grid_cell = float(os.environ.get("CELL", "1.25"))
h = C.c_void_p()
L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
HTH = np.zeros(78); HTh = np.zeros(12); m = C.c_int64()
buf = (C.c_ulonglong * 16)()
lib.slio_dbg_tile_stats(buf, 1)
lib.slio_profile(h, 1)
L.check(lib.slio_iterate(h, C.byref(pose), 1, 0, L.dptr(HTH), L.dptr(HTh), C.byref(m)), "it")
ms = C.c_double(); n = C.c_int64()
lib.slio_profile_read(h, 0, C.byref(ms), C.byref(n))
lib.slio_dbg_tile_stats(buf, 0)
v = list(buf)
ok = max(v[0], 1)
print(f"cell {p.grid_cell} search {ms.value * 1e3:.1f} us  stages ok {v[0]} fail rows {v[1]} ent {v[2]} "
      f"pts {v[3]}  batches {v[9]}  tile queries {v[4]} global {v[5]}  mean rows {v[6] / ok:.1f} "
      f"ent {v[7] / ok:.1f} pts {v[8] / ok:.1f}", flush=True)
lib.slio_destroy(h)
