"""Where the fused pass's tail goes (diagnostic build: bash scripts/build_variant.sh
sstamp -DSLIO_SOLVE_STAMP, then python scripts/variant.py <that .so> scripts/tail_stamps.py).
C2 problem, fixed-mode device updates (every pass fused); the stamps of the
update's last pass: launch start (block 0), then the final workgroup's
partial issued / segment arrival / row stored / row arrival, the 64 rows
summed into super rows with the control block staged (one batch over all
threads), filter step chain, end.  Medians over the updates, microseconds."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

lib = L.load()
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
names = [("launch->final's partial", 20, 16), ("segment arrival", 16, 17), ("row sum + store", 17, 18),
         ("row arrival", 18, 19), ("rows + block staged", 19, 4), ("S, w", 4, 9), ("cholesky + solves", 9, 10),
         ("dx + ballot", 10, 11), ("boxplus", 11, 12), ("flags -> P update / end", 12, 8)]
acc = {m: [] for m in (1, 2, 4)}
for rep in range(14):
    for maxit in (1, 2, 4):
        xs = L.SlioState()
        xs.pos[:] = list(st0[0:3]); xs.rot[:] = list(st0[3:7]); xs.rli[:] = list(st0[7:11])
        xs.tli[:] = list(st0[11:14]); xs.grav[:] = list(st0[23:26])
        P = np.eye(24) * 1e-2
        stt = L.SlioIkfStats()
        L.check(lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, maxit, 0, L.SLIO_MODE_FIXED,
                                           L.ALLREDUCE_FN(), None, C.byref(stt)), "ikf")
        buf = (C.c_ulonglong * 32)()
        lib.slio_dbg_solve_stamps(buf)
        if rep >= 2:
            acc[maxit].append(np.array(buf[:32], dtype=np.int64))
for maxit in (1, 2, 4):
    d = np.array(acc[maxit])
    parts = [f"{n}={np.median(d[:, b] - d[:, a]) * 0.01:.2f}" for n, a, b in names]
    print(f"maxit {maxit} (last pass): " + "  ".join(parts) + f"  total={np.median(d[:, 8] - d[:, 20]) * 0.01:.2f}")
# fixed mode, maxit 4: per pass k, block 0's start [21 + k + 1 & 3] and the filter step's end
# [25 + ...]: the pass's span and the boundary to the next pass's start
d = np.array(acc[4])
st = [d[:, 21 + ((k + 1) & 3)] for k in range(4)]
en = [d[:, 25 + ((k + 1) & 3)] for k in range(4)]
spans = [f"{np.median(en[k] - st[k]) * 0.01:.2f}" for k in range(4)]
gaps = [f"{np.median(st[k + 1] - en[k]) * 0.01:.2f}" for k in range(3)]
print(f"maxit 4 per pass: span (block 0 start -> filter step end) {spans}; end -> next pass's block 0 start {gaps}")
lib.slio_destroy(h)
