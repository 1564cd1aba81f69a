"""Per-block phase stamps (SLIO_ABL_STAMP build) of the LAST pass of the C2
update, kNN certificates on and off: start spread, kNN fast path (per wave),
refinement, fit, products; medians and the span.
  OUT=_var bash scripts/build_variant.sh STAMP -DSLIO_ABL_STAMP
  SLIO_LIB=_var/libslio_STAMP.so python scripts/stamps_cert.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402
from variant import use  # noqa: E402

lib = use(os.environ["SLIO_LIB"])
lib.slio_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
p = L.SlioParams(); lib.slio_params_default(C.byref(p))
h = C.c_void_p(); L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
bx, by, bz = (np.ascontiguousarray(body[:, k]) for k in range(3))
L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), body.shape[0]), "scan")
st0 = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9), [0, 0, -9.81]])
nb = (body.shape[0] + 127) // 128
for env in ("1", "0", "1", "0"):
    os.environ["SLIO_NO_KNN_CERT"] = env
    lib.slio_debug_reload_switches(h)
    for it in (2, 3, 4):
        for rep in range(3):
            xs = L.SlioState()
            xs.pos[:] = list(st0[0:3]); xs.rot[:] = list(st0[3:7]); xs.rli[:] = list(st0[7:11])
            xs.tli[:] = list(st0[11:14]); xs.grav[:] = list(st0[23:26])
            P = np.eye(24) * 1e-2
            st = L.SlioIkfStats()
            L.check(lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, it, 0, L.SLIO_MODE_FIXED,
                                               L.ALLREDUCE_FN(), None, C.byref(st)), "ikf")
        buf = (C.c_ulonglong * (8 * nb))()
        assert lib.slio_debug_stamps(buf, nb) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
        us = (a - a[:, 0].min()) / 100.0
        knn = us[:, 4:8].max(1) - us[:, 0]
        print(f"cert {'off' if env == '1' else 'on '} pass {it - 1}: start p50 {np.median(us[:, 0]):5.1f} max "
              f"{us[:, 0].max():5.1f} | knn p50 {np.median(knn):5.1f} max {knn.max():5.1f} | refine p50 "
              f"{np.median(us[:, 1] - us[:, 4:8].max(1)):4.1f} | fit p50 {np.median(us[:, 2] - us[:, 1]):4.1f} | "
              f"prod p50 {np.median(us[:, 3] - us[:, 2]):4.1f} | end p50 {np.median(us[:, 3]):5.1f} max "
              f"{us[:, 3].max():5.1f}")
lib.slio_destroy(h)
