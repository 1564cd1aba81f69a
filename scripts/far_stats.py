"""Diagnostic: far-queue use and search-pass time per synthetic problem.
usage: python scripts/far_stats.py N_MAP SENSOR [N_MAP SENSOR ...]"""
import ctypes as C
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402
from test_gpu_parity import iterate, mk, state_of, upload_map, upload_scan  # noqa: E402

lib = L.load()
args = sys.argv[1:]
for k in range(0, len(args), 2):
    n_map, sensor = int(args[k]), args[k + 1]
    t0 = time.time()
    mp, fr = synth.make_problem(n_map, 100_000, pattern="avia", sensor=sensor, cache_dir="/tmp/slio_cache")
    body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
    tg = time.time() - t0
    h = mk(L, cell=1.25)
    upload_map(L, h, mp)
    upload_scan(L, h, body)
    st = state_of(fr)
    for _ in range(3):
        iterate(L, h, st, True)
    lib.slio_profile(h, 1)
    for _ in range(20):
        iterate(L, h, st, True)
    ms, nl = C.c_double(), C.c_int64()
    lib.slio_profile_read(h, L.SLIO_KERNEL_SEARCH, C.byref(ms), C.byref(nl))
    ms2, nl2 = C.c_double(), C.c_int64()
    lib.slio_profile_read(h, L.SLIO_KERNEL_SUPER, C.byref(ms2), C.byref(nl2))
    nfar = C.c_int64()
    rc = lib.slio_far_queries(h, C.byref(nfar))
    print(json.dumps({"map": n_map, "sensor": sensor, "gen_s": round(tg, 1), "far": nfar.value, "far_rc": rc,
                      "search_us": 1e3 * ms.value / max(nl.value, 1),
                      "super_us": 1e3 * ms2.value / max(nl2.value, 1)}), flush=True)
    lib.slio_destroy(h)
