"""Diagnostic: tiny maps through the far queue, one case at a time, with the
far-queue error words checked after every pass (slio_far_queries)."""
import ctypes as C
import sys
import time

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from agi_lidar_slam_amd import _lib as L  # noqa: E402
from test_gpu_parity import IDENT, iterate, mk, results, upload_map, upload_scan  # noqa: E402

import os  # noqa: E402
lib = L.load(os.environ.get("SLIO_LIB", L.LIB_PATH))
print("lib", os.environ.get("SLIO_LIB", L.LIB_PATH), flush=True)
rng = np.random.default_rng(9)
for npts, nq in [(1, 1), (1, 64), (1, 300), (7, 300), (200, 3000)]:
    mp = rng.uniform(-3, 3, (npts, 3)).astype(np.float32)
    q = rng.uniform(-10, 10, (nq, 3)).astype(np.float32)
    h = mk(L, cell=1.0, n_max=nq)
    upload_map(L, h, mp)
    upload_scan(L, h, q)
    t0 = time.time()
    pose = L.SlioPose()
    pose.rot[:] = [1, 0, 0, 0]
    pose.rli[:] = [1, 0, 0, 0]
    rc = lib.slio_iterate_async(h, C.byref(pose), 1, 0, None)
    n = C.c_int64()
    rc2 = lib.slio_far_queries(h, C.byref(n))
    print(f"npts {npts} nq {nq}: launch rc {rc} far rc {rc2} far {n.value} "
          f"err {lib.slio_last_error()} {time.time() - t0:.3f}s", flush=True)
    idx, sqd, *_ = results(L, h, nq)
    d = (q[:, None, :] - mp[None]) ** 2
    d32 = (d[..., 0] + d[..., 1]) + d[..., 2]
    k = min(5, npts)
    ok = np.array_equal(np.sort(d32, 1)[:, :k], sqd[:, :k])
    print("   match", ok, flush=True)
    lib.slio_destroy(h)
