"""Per-block phase stamps of the LAST search pass of a device-resident C2
update (fixed mode, 4 IKF iterations from the initial pose), from the
SLIO_ABL_STAMP diagnostic build: shows the chunk order's effect (passes
after the first take chunks in chunk_order's order).  Blocks are indexed by
blockIdx (block b runs on CU b mod 256)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

from variant import use  # noqa: E402
lib = use(os.environ.get("SLIO_LIB", os.path.join(os.path.dirname(L.LIB_PATH), "_abl", "libslio_STAMP.so")))
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
for it in (1, 4):
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
    tot = us[:, 3] - us[:, 0]
    cu = np.arange(nb) % 256
    ends = np.array([us[cu == c, 3].max() for c in range(256)])
    tag = "pass 0 (index order)" if it == 1 else "pass 3 (chunk order)"
    print(f"{tag}: span {us[:, 3].max():.1f} us; CU end mean {ends.mean():.1f} p90 {np.quantile(ends, .9):.1f} "
          f"max {ends.max():.1f}; block total p50 {np.median(tot):.1f} max {tot.max():.1f}; "
          f"blocks >= 768 end {np.round(us[768:, 3], 1).tolist()}")
    np.savez(f"gpurun_out/stamps_update_it{it}.npz", stamps=a)
lib.slio_destroy(h)
