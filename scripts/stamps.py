"""Per-block phase timing from the SLIO_ABL_STAMP diagnostic build."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

from variant import use  # noqa: E402
lib = use(os.environ.get("SLIO_LIB", os.path.join(os.path.dirname(L.LIB_PATH), "_abl", "libslio_STAMP.so")))
lib.slio_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
for lpq in [int(v) for v in os.environ.get("LPQS", "102,2").split(",")]:
    for nscan in [100000]:
        mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
        body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)][:nscan])
        at_gt = os.environ.get("STAMP_POSE", "init") == "gt"
        st = np.concatenate([fr.gt_pos if at_gt else fr.init_pos, fr.gt_rot if at_gt else fr.init_rot,
                             [1, 0, 0, 0], synth.AVIA_T_LI])
        pose = L.SlioPose()
        pose.pos[:] = list(st[0:3]); pose.rot[:] = list(st[3:7])
        pose.rli[:] = list(st[7:11]); pose.tli[:] = list(st[11:14])
        p = L.SlioParams(); lib.slio_params_default(C.byref(p)); p.grid_cell = float(os.environ.get("STAMP_CELL", "0")); p.lanes_per_query = lpq
        h = C.c_void_p(); L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
        x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
        L.check(lib.slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
        bx, by, bz = (np.ascontiguousarray(body[:, k]) for k in range(3))
        L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), body.shape[0]), "scan")
        HTH = np.zeros(78); HTh = np.zeros(12); m = C.c_int64()
        for _ in range(5):
            L.check(lib.slio_iterate(h, C.byref(pose), 1, 0, L.dptr(HTH), L.dptr(HTh), C.byref(m)), "it")
        nb = (nscan + 127) // 128
        buf = (C.c_ulonglong * (8 * nb))()
        assert lib.slio_debug_stamps(buf, nb) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
        hw = (C.c_uint32 * (2 * nb))()
        lib.slio_debug_hwid.argtypes = [C.POINTER(C.c_uint32), C.c_int]
        assert lib.slio_debug_hwid(hw, nb) == 0
        ws = (C.c_ulonglong * (16 * nb))()
        lib.slio_debug_wstamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
        assert lib.slio_debug_wstamps(ws, nb) == 0
        rs = (C.c_ulonglong * (4 * nb))()
        lib.slio_debug_rstamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
        assert lib.slio_debug_rstamps(rs, nb) == 0
        rsa = np.frombuffer(rs, dtype=np.uint64).reshape(nb, 4).astype(np.int64)
        os.makedirs("gpurun_out", exist_ok=True)
        np.savez(f"gpurun_out/stamps_{lpq}_{nscan}.npz", stamps=a,
                 hwid=np.frombuffer(hw, dtype=np.uint32).reshape(nb, 2),
                 wstamps=np.frombuffer(ws, dtype=np.uint64).reshape(nb, 4, 4), rstamps=rsa)
        t0 = a[:, 0].min()
        us = (a - t0) / 100.0   # 100 MHz -> us
        ph1 = us[:, 1] - us[:, 0]; ph2 = us[:, 2] - us[:, 1]; ph3 = us[:, 3] - us[:, 2]
        wv = us[:, 4:8] - us[:, [0]]
        print(f"lpq={lpq} n={nscan} blocks={nb}: kernel span {us[:, 3].max():.1f}us; start spread {us[:, 0].max():.1f}us")
        for name, v in (("knn", ph1), ("fit", ph2), ("prod", ph3)):
            print(f"  {name}: mean {v.mean():.2f} p50 {np.median(v):.2f} p90 {np.quantile(v, .9):.2f} max {v.max():.2f} us")
        print(f"  wave kNN end: mean {wv.mean():.2f} max {wv.max():.2f}; per-block max-min wave {np.mean(wv.max(1) - wv.min(1)):.2f} us")
        tot = us[:, 3] - us[:, 0]
        print(f"  block total: p10 {np.quantile(tot, .1):.1f} p50 {np.median(tot):.1f} p90 {np.quantile(tot, .9):.1f} max {tot.max():.1f}; "
              f"end times p50 {np.median(us[:, 3]):.1f} p90 {np.quantile(us[:, 3], .9):.1f}")
        wsa = np.frombuffer(ws, dtype=np.uint64).reshape(nb, 4, 4).astype(np.int64)
        nref = wsa[:, :, 3]   # refining queries per wave (WSTAMP(3))
        rdur = (wsa[:, :, 1] - wsa[:, :, 0]) / 100.0
        print(f"  refining queries per wave: mean {nref.mean():.2f} p90 {np.quantile(nref, .9):.0f} max {nref.max()}; "
              f"waves with any {np.mean(nref > 0):.3f}; total {nref.sum()}")
        print(f"  refine duration per wave: mean {rdur.mean():.2f} p90 {np.quantile(rdur, .9):.2f} max {rdur.max():.2f} us")
        bref = nref.sum(1)
        one = np.nonzero((bref >= 1) & (bref <= 4) & (rsa[:, 0] > 0))[0]
        if one.size:
            seg = np.diff(rsa[one], axis=1) / 100.0
            st = (rsa[one, 0] - wsa[one, 0, 0]) / 100.0
            en = (wsa[one, 0, 1] - rsa[one, 3]) / 100.0
            print(f"  wide refine (blocks with 1-4 refs, n={one.size}): start->entry {st.mean():.2f}, bounds {seg[:, 0].mean():.2f}, "
                  f"table {seg[:, 1].mean():.2f}, scan {seg[:, 2].mean():.2f}, merge+write+sync {en.mean():.2f} us")
        slow = np.argsort(-tot)[:5]
        for b in slow:
            print(f"    slow block {b}: total {tot[b]:.1f} knn {ph1[b]:.1f} fit {ph2[b]:.1f} refs/wave {[int(v) for v in nref[b]]} "
                  f"refine us {[round(float(v), 1) for v in rdur[b]]}")
        lib.slio_destroy(h)
