"""Per-pass phases of a device-resident C2 update (fixed flow, 4 passes) from
the in-kernel stamps of a -DSLIO_SOLVE_STAMP build: block 0's start of pass k,
the final workgroup's last row arrival (every chunk of the pass done), the
filter step's end, and the gap to block 0's start of pass k + 1 -- for the
persistent update (SLIO_PERSIST=1) and a launch per pass (the default).

  OUT=_var bash scripts/build_variant.sh sstamp -DSLIO_SOLVE_STAMP
  SLIO_LIB=_var/libslio_sstamp.so python scripts/persist_stamps.py [CFG ...]   (CFG: - or K=V,K=V)
"""
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
fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
p = L.SlioParams()
lib.slio_params_default(C.byref(p))
h = C.c_void_p()
L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
st0 = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9), [0, 0, -9.81]])
CFGS = sys.argv[1:] or ["SLIO_PERSIST=1", "-"]
KEYS = sorted({kv.split("=")[0] for c in CFGS if c != "-" for kv in c.split(",")})
for cfg in CFGS:
    for k in KEYS:
        os.environ.pop(k, None)
    if cfg != "-":
        for kv in cfg.split(","):
            k, v = kv.split("=")
            os.environ[k] = v
    lib.slio_debug_reload_switches(h)
    rows = []
    for rep in range(40):
        xs = L.SlioState()
        xs.pos[:] = list(st0[0:3]); xs.rot[:] = list(st0[3:7]); xs.rli[:] = list(st0[7:11])
        xs.tli[:] = list(st0[11:14]); xs.grav[:] = list(st0[23:26])
        P = np.eye(24) * 1e-2
        st = L.SlioIkfStats()
        L.check(lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, 4, 0, 1,
                                           L.ALLREDUCE_FN(), None, C.byref(st)), "ikf")
        buf = (C.c_ulonglong * 64)()
        lib.slio_dbg_solve_stamps(buf)
        v = np.array(buf[:], dtype=np.int64)
        k = [(q + 1) & 3 for q in range(4)]
        start = v[[21 + i for i in k]]
        last = v[[32 + i for i in k]]
        end = v[[25 + i for i in k]]
        wait = v[[40 + i for i in k]]
        # the last pass's tail: last row arrival -> staged, step start, chain
        # done, P updated, end (SSTAMP 4, 5, 6, 7 of its filter step)
        tl = v[[4, 5, 6, 7]] - last[3]
        if rep >= 5:
            rows.append(np.concatenate([last - start, end - last, np.append(start[1:] - end[:-1], 0),
                                        np.append(start[1:] - wait[1:], 0), tl, [end[-1] - start[0]]]) * 10)
    d = np.median(np.array(rows), axis=0) / 1e3  # 100 MHz ticks -> us
    path = lib.slio_debug_update_path(h)
    print(f"{cfg} (path {path}): total {d[-1]:.2f} us")
    for q in range(4):
        print(f"  pass {q}: search {d[q]:6.2f}  tail {d[4 + q]:5.2f}  gap->next {d[8 + q]:5.2f}"
              f"  block0 waited {d[12 + q]:5.2f}")
    print("  last tail from the last row arrival: staged %.2f  step start %.2f  chain done %.2f  P %.2f" %
          tuple(d[16:20]))
lib.slio_destroy(h)
