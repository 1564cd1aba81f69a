"""Bisect: reference-flow fused updates on fresh handles (one per scenario)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

lib = L.load()
mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
st0 = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9), [0, 0, -9.81]])
base = C.c_void_p()
p = L.SlioParams()
lib.slio_params_default(C.byref(p))
L.check(lib.slio_create(C.byref(base), C.byref(p)), "create")
x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
L.check(lib.slio_map_upload(base, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))


def upd(h, mode, maxit):
    xs = L.SlioState()
    xs.pos[:] = list(st0[0:3]); xs.rot[:] = list(st0[3:7]); xs.rli[:] = list(st0[7:11])
    xs.tli[:] = list(st0[11:14]); xs.grav[:] = list(st0[23:26])
    P = np.eye(24) * 1e-2
    stt = L.SlioIkfStats()
    rc = lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, maxit, 0, mode, L.ALLREDUCE_FN(), None,
                                    C.byref(stt))
    return rc, (lib.slio_last_error().decode() if rc else ""), (stt.passes, stt.searches, stt.converged)


for name, env_first, env_rest, mode, maxit, n in [
        ("ref3 fused", {}, {}, 0, 3, 40), ("ref4 fused", {}, {}, 0, 4, 40), ("fix4 fused", {}, {}, 1, 4, 40),
        ("ref3 nofuse0", {"SLIO_NO_FUSE0": "1"}, {"SLIO_NO_FUSE0": "1"}, 0, 3, 6),
        ("ref3 first nofuse", {"SLIO_NO_FUSE": "1"}, {}, 0, 3, 40),
        ("ref1 fused", {}, {}, 0, 1, 6), ("ref2 fused", {}, {}, 0, 2, 6)]:
    h = C.c_void_p()
    L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
    L.check(lib.slio_map_share(h, base), "share")
    L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
    out = []
    for k in range(n):
        env = env_first if k == 0 else env_rest
        for key in ("SLIO_NO_FUSE", "SLIO_NO_FUSE0"):
            os.environ.pop(key, None)
        os.environ.update(env)
        out.append(upd(h, mode, maxit))
    for key in ("SLIO_NO_FUSE", "SLIO_NO_FUSE0"):
        os.environ.pop(key, None)
    fails = [k for k, o in enumerate(out) if o[0]]
    print(name, "updates", len(out), "failed", fails, "stats", sorted(set(o[2] for o in out)), flush=True)
    lib.slio_destroy(h)
lib.slio_destroy(base)
