"""Diagnostic (SLIO_FAR_TRACE build): one tiny pass, far-queue events read
from mapped host memory while the kernel runs."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from agi_lidar_slam_amd import _lib as L  # noqa: E402

lib = L.load(os.environ["SLIO_LIB"])
hip = C.CDLL("libamdhip64.so")
buf = C.c_void_p()
assert hip.hipHostMalloc(C.byref(buf), C.c_size_t(4 * 4 * 4100), 0x2 | 0x40000000) == 0  # mapped | coherent
C.memset(buf, 0, 4 * 4 * 4100)
assert lib.slio_dbg_far_trace(buf) == 0
from test_gpu_parity import mk, upload_map, upload_scan  # noqa: E402
rng = np.random.default_rng(9)
npts, nq = int(sys.argv[1]), int(sys.argv[2])
mp = rng.uniform(-3, 3, (npts, 3)).astype(np.float32)
q = rng.uniform(-10, 10, (nq, 3)).astype(np.float32)
h = mk(L, cell=1.0, n_max=nq)
upload_map(L, h, mp)
upload_scan(L, h, q)
pose = L.SlioPose()
pose.rot[:] = [1, 0, 0, 0]
pose.rli[:] = [1, 0, 0, 0]
print("launch", lib.slio_iterate_async(h, C.byref(pose), 1, 0, None), flush=True)
arr = (C.c_uint32 * (4 * 4100)).from_address(buf.value)
time.sleep(3)
n = min(arr[0], 4095)
print("events", arr[0], flush=True)
for k in range(n):
    r = arr[4 + 4 * k: 8 + 4 * k]
    print(f"blk {r[0] >> 8} wave {r[0] & 255}: ev {r[1]} {r[2]} {r[3]}", flush=True)
sys.stdout.flush()
os._exit(0)
