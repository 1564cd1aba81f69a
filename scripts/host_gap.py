"""Where a C2 step's time goes on the host side, and how step times evolve
after an idle period (the driver's bench setting is --steps 20 --warmup 5).

bench.py's C2 setup and step, with the library's host stamps on
(slio_debug_host_stamps): per update the Python call overhead, the library's
set-up, the first launch, the remaining launches, the wait for the published
result and the return.  `wait` (first launch enqueued -> result seen) minus
the kernels' own time (rocprofv3) is the dispatch + publication latency.

  python scripts/host_gap.py [--steps 300] [--idle 2.0]
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
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--idle", type=float, default=2.0)
    ap.add_argument("--series", type=int, default=60)
    args = ap.parse_args()
    from agi_lidar_slam_amd import _lib as L, synth
    lib = L.load()
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
    P_ptr, xs_ref, st_ref = L.dptr(P), C.byref(xs), C.byref(stats)
    fn = lib.slio_ikf_update_device
    hs = np.zeros(8, np.int64)
    hs_ptr = L.i64ptr(hs)

    def step():
        C.memmove(C.addressof(xs), C.addressof(xs0), C.sizeof(xs))
        P[...] = P0
        rc = fn(h, xs_ref, P_ptr, 0.001, 4, 0, L.SLIO_MODE_FIXED, cb, None, st_ref)
        if rc:
            L.check(rc, "ikf")

    def series(n, stamps):
        lib.slio_debug_host_stamps(h, 1 if stamps else 0, None)
        t = np.zeros(n + 1, np.int64)
        rows = []
        t[0] = time.perf_counter_ns()
        for k in range(n):
            a = time.perf_counter_ns()
            step()
            b = time.perf_counter_ns()
            t[k + 1] = b
            if stamps:
                lib.slio_debug_host_stamps(h, -1, hs_ptr)
                rows.append([a, *hs[:7], b])
        lib.slio_debug_host_stamps(h, 0, None)
        return np.diff(t) / 1e3, np.array(rows, np.int64)

    out = {}
    # bench.py's order: 5 warmup steps, then the timed ones
    d, _ = series(5, False)
    out["warmup_us"] = d.round(1).tolist()
    d, _ = series(20, False)
    out["first20_us"] = d.round(1).tolist()
    out["first20_mean_us"] = float(d.mean())
    d, _ = series(args.steps, False)
    out["steady_median_us"] = float(np.median(d))
    out["steady_mean_us"] = float(d.mean())
    # after an idle period
    time.sleep(args.idle)
    d, _ = series(args.series, False)
    out[f"after_{args.idle}s_idle_us"] = d.round(1).tolist()
    # stamps
    _, r = series(args.steps, True)
    # columns: py_call, s0 entry, s1 setup, s2 block ready, s3 launch0, s4 all launched, s5 seen, s6 exit, py_ret
    iv = {
        "py_call->entry": r[:, 1] - r[:, 0],
        "entry->setup": r[:, 2] - r[:, 1],
        "setup->block_ready": r[:, 3] - r[:, 2],
        "block_ready->launch0_returned": r[:, 4] - r[:, 3],
        "launch0->all_launched": r[:, 5] - r[:, 4],
        "all_launched->result_seen": r[:, 6] - r[:, 5],
        "launch0->result_seen": r[:, 6] - r[:, 4],
        "result_seen->exit": r[:, 7] - r[:, 6],
        "exit->py_return": r[:, 8] - r[:, 7],
        "py_return->next_py_call": r[1:, 0] - r[:-1, 8],
        "result_seen->next_launch0": r[1:, 4] - r[:-1, 6],
        "step": r[1:, 0] - r[:-1, 0],
    }
    out["stamps_median_us"] = {k: round(float(np.median(v)) / 1e3, 2) for k, v in iv.items()}
    out["stamps_p10_us"] = {k: round(float(np.percentile(v, 10)) / 1e3, 2) for k, v in iv.items()}
    print(json.dumps(out, indent=1))
    lib.slio_destroy(h)


if __name__ == "__main__":
    main()
