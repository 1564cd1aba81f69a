"""Drive the C2 search pass REPS times (for rocprofv3 PMC / ablation runs).
Env: SLIO_LIB (library path), LPQ, CELL, REPS, MODE (pass: slio_iterate at the
initial pose; update: bench.py's step, slio_ikf_update_device in fixed mode,
4 fused passes)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402


def main():
    from variant import use
    lib = use(os.environ["SLIO_LIB"]) if "SLIO_LIB" in os.environ else L.load()
    lpq = int(os.environ.get("LPQ", "2"))
    cell = float(os.environ.get("CELL", "1.0"))
    reps = int(os.environ.get("REPS", "20"))
    mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
    nscan = int(os.environ.get("NSCAN", "100000"))
    if os.environ.get("ORDER", "voxel") == "voxel":
        fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
    fr.body = np.ascontiguousarray(fr.body[:nscan])
    st = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI])
    pose = L.SlioPose()
    pose.pos[:] = list(st[0:3]); pose.rot[:] = list(st[3:7])
    pose.rli[:] = list(st[7:11]); pose.tli[:] = list(st[11:14])
    p = L.SlioParams()
    lib.slio_params_default(C.byref(p))
    p.grid_cell, p.lanes_per_query = cell, lpq
    p.search_radius = float(os.environ.get("RADIUS", "0.0"))
    h = C.c_void_p()
    L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
    x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
    L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
    bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
    L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
    HTH = np.zeros(78); HTh = np.zeros(12); m = C.c_int64()
    if os.environ.get("MODE", "pass") == "update":
        st0 = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9), [0, 0, -9.81]])
        stats = L.SlioIkfStats()
        cb = L.ALLREDUCE_FN()

        def upd():
            xs = L.SlioState()
            xs.pos[:] = list(st0[0:3]); xs.rot[:] = list(st0[3:7]); xs.rli[:] = list(st0[7:11])
            xs.tli[:] = list(st0[11:14]); xs.grav[:] = list(st0[23:26])
            P = np.eye(24) * 1e-2
            L.check(lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, 4, 0, L.SLIO_MODE_FIXED, cb, None,
                                               C.byref(stats)), "ikf")
        for _ in range(3):
            upd()
        lib.slio_profile(h, 1)
        t0 = time.perf_counter()
        for _ in range(reps):
            upd()
        el = (time.perf_counter() - t0) / reps
        ms = C.c_double(); n = C.c_int64()
        lib.slio_profile_read(h, 0, C.byref(ms), C.byref(n))
        print(json.dumps({"mode": "update", "search_us": ms.value / n.value * 1e3, "update_wall_us": el * 1e6,
                          "m": stats.last_m}), flush=True)
        lib.slio_destroy(h)
        return
    for _ in range(3):
        L.check(lib.slio_iterate(h, C.byref(pose), 1, 0, L.dptr(HTH), L.dptr(HTh), C.byref(m)), "it")
    lib.slio_profile(h, 1)
    t0 = time.perf_counter()
    for _ in range(reps):
        L.check(lib.slio_iterate(h, C.byref(pose), 1, 0, L.dptr(HTH), L.dptr(HTh), C.byref(m)), "it")
    el = (time.perf_counter() - t0) / reps
    ms = C.c_double(); n = C.c_int64()
    lib.slio_profile_read(h, 0, C.byref(ms), C.byref(n))
    print(json.dumps({"lib": os.path.basename(os.environ.get("SLIO_LIB", "libslio.so")), "lpq": lpq,
                      "cell": cell, "radius": p.search_radius, "nscan": nscan, "search_us": ms.value / n.value * 1e3,
                      "iter_wall_us": el * 1e6, "m": m.value}), flush=True)
    lib.slio_destroy(h)


if __name__ == "__main__":
    main()
