"""Per-workgroup timing of each pass of a device-resident C2 update (fixed
flow): the SLIO_ABL_STAMP build's per-block stamps (start, refinements done,
fit done, products done) of the last pass, collected with maximum_iter 1..4
so that each pass in turn is the last.  Shows how far the pass's end (its
slowest workgroup) lies beyond the typical workgroup: the load imbalance.

  OUT=_var bash scripts/build_variant.sh STAMP -DSLIO_ABL_STAMP
  SLIO_LIB=_var/libslio_STAMP.so python scripts/wg_stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

from variant import use  # noqa: E402
lib = use(os.environ["SLIO_LIB"])
lib.slio_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
lib.slio_debug_wstamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
lib.slio_debug_fstamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
lib.slio_debug_rstamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
lib.slio_debug_hwid.argtypes = [C.POINTER(C.c_uint32), C.c_int]
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
nb = (fr.body.shape[0] + 127) // 128
os.makedirs("gpurun_out", exist_ok=True)
for maxit in (1, 2, 3, 4):
    res = []
    for rep in range(6):
        xs = L.SlioState()
        xs.pos[:] = list(st0[0:3]); xs.rot[:] = list(st0[3:7]); xs.rli[:] = list(st0[7:11])
        xs.tli[:] = list(st0[11:14]); xs.grav[:] = list(st0[23:26])
        P = np.eye(24) * 1e-2
        st = L.SlioIkfStats()
        L.check(lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, maxit, 0, 1,
                                           L.ALLREDUCE_FN(), None, C.byref(st)), "ikf")
        buf = (C.c_ulonglong * (8 * nb))()
        assert lib.slio_debug_stamps(buf, nb) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
        ws = (C.c_ulonglong * (16 * nb))()
        assert lib.slio_debug_wstamps(ws, nb) == 0
        wsa = np.frombuffer(ws, dtype=np.uint64).reshape(nb, 4, 4).astype(np.int64)
        fs = (C.c_ulonglong * (6 * nb))()
        assert lib.slio_debug_fstamps(fs, nb) == 0
        fsa = np.frombuffer(fs, dtype=np.uint64).reshape(nb, 6).astype(np.int64)
        rs = (C.c_ulonglong * (6 * nb))()
        assert lib.slio_debug_rstamps(rs, nb) == 0
        rsa = np.frombuffer(rs, dtype=np.uint64).reshape(nb, 6).astype(np.int64)
        lib.slio_debug_clear_stamps()
        hw = (C.c_uint32 * (2 * nb))()
        assert lib.slio_debug_hwid(hw, nb) == 0
        hwa = np.frombuffer(hw, dtype=np.uint32).reshape(nb, 2).astype(np.int64)
        res.append((a, wsa, fsa, rsa, hwa))
    a, wsa, fsa, rsa, hwa = res[-1]
    fd = np.diff(fsa[:, :5], axis=1) / 100.0
    far = (fsa[:, 0] - a[:, 1]) / 100.0
    np.savez(f"gpurun_out/wg_stamps_pass{maxit - 1}.npz", stamps=a, wstamps=wsa, fstamps=fsa, rstamps=rsa)
    t0 = a[:, 0].min()
    us = (a - t0) / 100.0
    tot = us[:, 3] - us[:, 0]
    knn = us[:, 1] - us[:, 0]
    fit = us[:, 2] - us[:, 1]
    prod = us[:, 3] - us[:, 2]
    nref = wsa[:, :, 3].sum(1)
    print(f"pass {maxit - 1}: span {us[:, 3].max():.1f} us; starts p50 {np.median(us[:, 0]):.2f} max {us[:, 0].max():.2f}")
    print(f"  WG total p10 {np.quantile(tot, .1):.1f} p50 {np.median(tot):.1f} mean {tot.mean():.1f} "
          f"p90 {np.quantile(tot, .9):.1f} p99 {np.quantile(tot, .99):.1f} max {tot.max():.1f}")
    print(f"  WG end p50 {np.median(us[:, 3]):.1f} p90 {np.quantile(us[:, 3], .9):.1f} "
          f"p99 {np.quantile(us[:, 3], .99):.1f} max {us[:, 3].max():.1f}")
    print(f"  phases p50/max: knn+refine {np.median(knn):.1f}/{knn.max():.1f}  fit {np.median(fit):.1f}/{fit.max():.1f}"
          f"  products {np.median(prod):.1f}/{prod.max():.1f}")
    print(f"  fit (wave 0): after-refine->fit entry p50 {np.median(far):.2f}; loads {np.median(fd[:, 0]):.2f}  "
          f"plane+gate {np.median(fd[:, 1]):.2f}  row+stores {np.median(fd[:, 2]):.2f}  lds+drain {np.median(fd[:, 3]):.2f}"
          f"  (p90 {np.quantile(fd[:, 0], .9):.2f} {np.quantile(fd[:, 1], .9):.2f} {np.quantile(fd[:, 2], .9):.2f}"
          f" {np.quantile(fd[:, 3], .9):.2f}); barrier after wave 0 {np.median(a[:, 2] / 100.0 - fsa[:, 4] / 100.0):.2f}")
    print(f"  refining queries per WG: mean {nref.mean():.1f} max {nref.max()}; corr(total, refs) "
          f"{np.corrcoef(tot, nref)[0, 1]:.2f}")
    for b in np.argsort(-tot)[:8]:
        r = rsa[b]
        rinfo = ""
        if r[0] > 0:
            rinfo = (f" | wide refine: cand {r[4]} runs {r[5] & 255} RL {(r[5] >> 8) & 255} finite {(r[5] >> 16) & 1}"
                     f" bounds {(r[1] - r[0]) / 100:.2f} table {(r[2] - r[1]) / 100:.2f} scan {(r[3] - r[2]) / 100:.2f} us")
        print(f"    slow WG {b}: start {us[b, 0]:.1f} total {tot[b]:.1f} knn {knn[b]:.1f} fit {fit[b]:.1f} "
              f"prod {prod[b]:.1f} refs {int(nref[b])}{rinfo}")
    # workgroups per CU (HW_ID cu / sh / se, XCC_ID) and the WG time by that count
    cu = (hwa[:, 1] & 0xF) * 4096 + ((hwa[:, 0] >> 8) & 0xF) * 64 + ((hwa[:, 0] >> 12) & 1) * 8 + ((hwa[:, 0] >> 13) & 7)
    _, inv, cnt = np.unique(cu, return_inverse=True, return_counts=True)
    per = cnt[inv]
    print("  WGs per CU: " + ", ".join(f"{k}: {int((cnt == k).sum())} CUs, WG total p50 {np.median(tot[per == k]):.1f} "
                                      f"max {tot[per == k].max():.1f}" for k in sorted(set(cnt.tolist()))))
    late = np.arange(nb) >= 768
    print(f"  blocks >= 768: per-CU count {np.bincount(per[late]).tolist()}; WG total p50 {np.median(tot[late]):.1f}")
    w = rsa[:, 0] > 0
    if w.any():
        c = rsa[w, 4]
        print(f"  wide refinements (thread 0, {w.sum()} WGs): candidates p50 {np.median(c):.0f} p90 "
              f"{np.quantile(c, .9):.0f} max {c.max()}; scan us p50 {np.median((rsa[w, 3] - rsa[w, 2]) / 100):.2f} "
              f"max {((rsa[w, 3] - rsa[w, 2]) / 100).max():.2f}; finite bound {np.mean((rsa[w, 5] >> 16) & 1):.2f}")
lib.slio_destroy(h)
