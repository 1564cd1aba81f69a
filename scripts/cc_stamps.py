"""Phase stamps of k_lego_cc (diagnostic build -DSLIO_FE_STAMP,
SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_fe.so) on the VLP-16 sweep."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402
from agi_lidar_slam_amd.lego import LegoFrontEnd, LegoParams  # noqa: E402

from variant import use  # noqa: E402
lib = use(os.environ["SLIO_LIB"])
lib.slio_dbg_cc_stamps.argtypes = [C.POINTER(C.c_ulonglong)]
sw = synth.make_vlp16_sweep()
fe = LegoFrontEnd(LegoParams())
fe.upload(sw["x"], sw["y"], sw["z"])
names = ["stage edges", "row runs", "unions", "roots", "sizes", "outputs"]
acc = []
for rep in range(20):
    fe.run()
    buf = (C.c_ulonglong * 8)()
    assert lib.slio_dbg_cc_stamps(buf) == 0
    acc.append(np.diff(np.array(buf[:7], dtype=np.int64)) / 100.0)
a = np.median(np.array(acc[5:]), axis=0)
for k, nm in enumerate(names):
    print(f"cc {nm:12s} {a[k]:6.2f} us")
print(f"cc total {a.sum():.2f} us")
fe.close()
