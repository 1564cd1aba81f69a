#!/usr/bin/env python3
"""In-process A/B of C2 update variants selected by environment switches the
library reads per update (SLIO_NO_FUSE, SLIO_NO_FUSE0, SLIO_NO_MFMA, ...):
one map, one scan, one handle; the configurations take turns in rounds of
--steps updates and each reports the median IKF it/s over the rounds (the
box-to-box and run-to-run spread of separate bench.py runs is ~2-3 %).

  python scripts/ab_inproc.py - SLIO_NO_FUSE=1 "SLIO_NO_MFMA=1,SLIO_NO_FUSE0=1"
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=4)
    args = ap.parse_args()
    from agi_lidar_slam_amd import _lib as L, synth
    lib = L.load()
    mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
    fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
    p = L.SlioParams()
    lib.slio_params_default(C.byref(p))
    p.max_points = 100_000
    h = C.c_void_p()
    L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
    x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
    L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
    bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
    L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
    st0 = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9), [0, 0, -9.81]])
    xs0 = L.SlioState()
    xs0.pos[:] = list(st0[0:3])
    xs0.rot[:] = list(st0[3:7])
    xs0.rli[:] = list(st0[7:11])
    xs0.tli[:] = list(st0[11:14])
    xs0.grav[:] = list(st0[23:26])
    xs = L.SlioState()
    P0 = np.eye(24) * 1e-2
    P = np.empty_like(P0)
    stats = L.SlioIkfStats()
    cb = L.ALLREDUCE_FN()
    keys = sorted({kv.split("=")[0] for c in args.configs if c != "-" for kv in c.split(",")})

    def set_env(cfg):
        for k in keys:
            os.environ.pop(k, None)
        if cfg != "-":
            for kv in cfg.split(","):
                k, v = kv.split("=")
                os.environ[k] = v
        lib.slio_debug_reload_switches(h)

    def run(n):
        for _ in range(n):
            C.memmove(C.addressof(xs), C.addressof(xs0), C.sizeof(xs))
            P[...] = P0
            rc = lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, args.iters, 0, L.SLIO_MODE_FIXED,
                                            cb, None, C.byref(stats))
            if rc:
                L.check(rc, "ikf")

    res = {c: [] for c in args.configs}
    for c in args.configs:
        set_env(c)
        run(10)
    for r in range(args.rounds):
        for c in args.configs:
            set_env(c)
            run(3)
            t0 = time.perf_counter()
            run(args.steps)
            el = time.perf_counter() - t0
            res[c].append(args.steps * args.iters / el)
    for c in args.configs:
        v = np.array(res[c])
        print(json.dumps({"config": c, "median_ikf_it_s": round(float(np.median(v))),
                          "us_per_step": round(1e6 * args.iters / float(np.median(v)), 1),
                          "min": round(float(v.min())), "max": round(float(v.max()))}), flush=True)
    lib.slio_destroy(h)


if __name__ == "__main__":
    main()
