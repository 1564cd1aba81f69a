"""Phase stamps of k_lio_features (debug build -DSLIO_LIO_STAMP,
SLIO_LIB=agi_lidar_slam_amd/_abl/libslio_lstamp.so), ring 32 of the C3 scan."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

lib = L.load(os.environ["SLIO_LIB"])
from agi_lidar_slam_amd.frontend import LioSamFrontEnd, LioSamParams, imu_deskew_table  # noqa: E402

lib.slio_dbg_lio_stamps.argtypes = [C.POINTER(C.c_ulonglong)]
sc = synth.make_ouster_scan()
tb = imu_deskew_table(sc["imu_stamps"], sc["imu_gyro"], sc["time_scan_cur"], sc["time_scan_end"])
fe = LioSamFrontEnd(LioSamParams(N_SCAN=64, Horizon_SCAN=2048))
fe.set_deskew(*tb[:4], sc["time_scan_cur"], tb[4])
fe.upload(sc["x"], sc["y"], sc["z"], sc["intensity"], sc["ring"], sc["time"])
acc = []
prev = None
for rep in range(12):
    fe.run()
    buf = (C.c_ulonglong * (256 * 8))()
    lib.slio_dbg_lio_stamps(buf)
    v = np.array(buf[:], dtype=np.int64).reshape(256, 8)[:64]
    if prev is not None and rep >= 3:
        ph = np.concatenate([np.diff(v[:, :6], axis=1), v[:, 6:8] - prev[:, 6:8]], axis=1) * 10
        acc.append(ph)
    prev = v
ph = np.median(np.array(acc), axis=0)  # (64 rings, 7 phases) ns
tot = ph[:, :5].sum(axis=1)
names = ["load+reach", "sort+picks", "corners+voxkeys", "voxel sort", "centroids", "sorts", "picks"]
for r in [int(np.argmax(tot)), 32, 0]:
    print(f"ring {r:2d} total {tot[r] / 1e3:6.1f} us  " +
          "  ".join(f"{n}={t / 1e3:.1f}" for n, t in zip(names, ph[r])))
print("rings by total (us):", np.round(np.sort(tot)[::-1][:8] / 1e3, 1))
fe.close()
