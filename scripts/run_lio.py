"""Time the LIO-SAM front-end on the C3 Ouster scan (inputs resident)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

from variant import use  # noqa: E402
use(os.environ["SLIO_LIB"]) if "SLIO_LIB" in os.environ else L.load()
from agi_lidar_slam_amd.frontend import LioSamFrontEnd, LioSamParams, imu_deskew_table  # noqa: E402

reps = int(os.environ.get("REPS", "200"))
sc = synth.make_ouster_scan()
tb = imu_deskew_table(sc["imu_stamps"], sc["imu_gyro"], sc["time_scan_cur"], sc["time_scan_end"])
fe = LioSamFrontEnd(LioSamParams(N_SCAN=64, Horizon_SCAN=2048))
fe.set_deskew(*tb[:4], sc["time_scan_cur"], tb[4])
fe.upload(sc["x"], sc["y"], sc["z"], sc["intensity"], sc["ring"], sc["time"])
for _ in range(5):
    fe.run()
t0 = time.perf_counter()
for _ in range(reps):
    fe.lib.slio_lio_run_async(fe.h)
c = fe.run()
el = time.perf_counter() - t0
print(f"{(reps + 1) / el:.1f} scans/s  {el / (reps + 1) * 1e6:.1f} us/scan  n_ext {c.n_extracted} "
      f"corner {c.n_corner} surface {c.n_surface}")
fe.close()
