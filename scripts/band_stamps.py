"""Phase stamps of k_lego_cc_band (diagnostic build -DSLIO_FE_STAMP; bind it
with SLIO_LIB=...) on the VLP-16 sweep: per band (median over bands) and the
last arriver's merge."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import synth  # noqa: E402
from agi_lidar_slam_amd.lego import LegoFrontEnd, LegoParams  # noqa: E402

from variant import use  # noqa: E402
lib = use(os.environ["SLIO_LIB"])
lib.slio_dbg_band_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]
sw = synth.make_vlp16_sweep()
fe = LegoFrontEnd(LegoParams())
fe.upload(sw["x"], sw["y"], sw["z"])
nb = (1800 + 63) // 64
res = []
for rep in range(30):
    fe.run()
    b = (C.c_ulonglong * (64 * 8))()
    m = (C.c_ulonglong * 8)()
    assert lib.slio_dbg_band_stamps(b, m) == 0
    a = np.array(b, dtype=np.int64).reshape(64, 8)[:nb, :7]
    mm = np.array(m, dtype=np.int64)[:5]
    t0 = a[:, 0].min()
    res.append(np.concatenate([np.median(a - t0, axis=0), [a[:, 6].max() - t0], mm - t0]) / 100.0)
r = np.median(np.array(res[5:]), axis=0)
names = ["start", "staged", "edges", "runs", "unions", "roots+counts", "arrived", "last arrival",
         "merge start", "init", "records", "unions", "end"]
for k, nm in enumerate(names):
    print(f"band {nm:14s} {r[k]:7.2f} us")
fe.close()
