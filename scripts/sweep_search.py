"""Sweep search-kernel variants (lanes per query x grid cell) on the C2
workload; prints avg k_search_pass time per variant (HIP events)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402


def main():
    lpqs = [int(v) for v in os.environ.get("LPQS", "1,2,4").split(",")]
    cells = [float(v) for v in os.environ.get("CELLS", "1.0,1.25,1.5").split(",")]
    reps = int(os.environ.get("REPS", "20"))
    lib = L.load()
    mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
    st = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI])
    pose = L.SlioPose()
    pose.pos[:] = list(st[0:3]); pose.rot[:] = list(st[3:7])
    pose.rli[:] = list(st[7:11]); pose.tli[:] = list(st[11:14])
    x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
    bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
    res = []
    ref = None
    for cell in cells:
        base = None
        for lpq in lpqs:
            p = L.SlioParams()
            lib.slio_params_default(C.byref(p))
            p.grid_cell, p.lanes_per_query = cell, lpq
            h = C.c_void_p()
            L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
            if base is None:
                L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
                base = h
            else:
                L.check(lib.slio_map_share(h, base), "share")
            L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
            HTH = np.zeros(78); HTh = np.zeros(12); m = C.c_int64()
            for _ in range(3):
                L.check(lib.slio_iterate(h, C.byref(pose), 1, 0, L.dptr(HTH), L.dptr(HTh), C.byref(m)), "it")
            if ref is None:
                ref = HTH.copy()
            assert np.allclose(HTH, ref, rtol=1e-9), "variant changed the result"
            lib.slio_profile(h, 1)
            t0 = time.perf_counter()
            for _ in range(reps):
                L.check(lib.slio_iterate(h, C.byref(pose), 1, 0, L.dptr(HTH), L.dptr(HTh), C.byref(m)), "it")
            el = (time.perf_counter() - t0) / reps
            ms = C.c_double(); n = C.c_int64()
            lib.slio_profile_read(h, 0, C.byref(ms), C.byref(n))
            ms2 = C.c_double(); n2 = C.c_int64()
            lib.slio_profile_read(h, 2, C.byref(ms2), C.byref(n2))
            r = {"cell": cell, "lpq": lpq, "search_us": ms.value / n.value * 1e3,
                 "super_us": ms2.value / n2.value * 1e3, "iter_wall_us": el * 1e6, "m": m.value}
            print(json.dumps(r), flush=True)
            res.append(r)
            lib.slio_profile(h, 0)
            if h is not base:
                lib.slio_destroy(h)
        lib.slio_destroy(base)
    best = min(res, key=lambda r: r["search_us"])
    print("BEST", json.dumps(best))


if __name__ == "__main__":
    main()
