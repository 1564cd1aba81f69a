"""Phase stamps of the fused super-sum + filter-step kernel (debug build with
-DSLIO_SOLVE_STAMP, SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_sstamp.so)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

from variant import use  # noqa: E402
lib = use(os.environ["SLIO_LIB"])
lib.slio_dbg_solve_stamps.argtypes = [C.POINTER(C.c_ulonglong)]
mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
p = L.SlioParams()
lib.slio_params_default(C.byref(p))
h = C.c_void_p()
L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
st0 = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9), [0, 0, -9.81]])
names = ["start", "-", "last-found", "-", "staged", "totals", "chain-done",
         "P", "end", "S+w", "chol+solve", "dx+ballot", "boxplus", "flags", "LM"]
acc = []
for rep in range(12):
    for maxit in (1, 2, 4):
        xs = L.SlioState()
        xs.pos[:] = list(st0[0:3]); xs.rot[:] = list(st0[3:7]); xs.rli[:] = list(st0[7:11])
        xs.tli[:] = list(st0[11:14]); xs.grav[:] = list(st0[23:26])
        P = np.eye(24) * 1e-2
        st = L.SlioIkfStats()
        L.check(lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, maxit, 0, 1,
                                           L.ALLREDUCE_FN(), None, C.byref(st)), "ikf")
        buf = (C.c_ulonglong * 32)()
        lib.slio_dbg_solve_stamps(buf)
        v = np.array(buf[:15], dtype=np.int64)
        if rep >= 2:
            acc.append((maxit, v - v[0]))
for maxit in (1, 2, 4):
    d = np.array([a for m, a in acc if m == maxit])
    med = np.median(d, axis=0) * 10  # wall_clock64: 100 MHz -> ns
    order = [0, 2, 4, 5, 9, 10, 11, 12, 13, 14, 6, 7, 8]
    print(f"maxit {maxit}: " + "  ".join(f"{names[k]}={med[k]/1e3:.2f}us" for k in order))
lib.slio_destroy(h)
