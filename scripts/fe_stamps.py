"""Phase stamps of k_fe_pick (diagnostic build -DSLIO_FE_STAMP,
SLIO_LIB=_var/libslio_fe.so, OUT=_var bash scripts/build_variant.sh fe -DSLIO_FE_STAMP) on the C3 scan."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402

from variant import use  # noqa: E402
lib = use(os.environ["SLIO_LIB"])
from agi_lidar_slam_amd.frontend import LioSamFrontEnd, LioSamParams, imu_deskew_table  # noqa: E402

lib.slio_dbg_fe_stamps.argtypes = [C.POINTER(C.c_ulonglong)]
sc = synth.make_ouster_scan()
tb = imu_deskew_table(sc["imu_stamps"], sc["imu_gyro"], sc["time_scan_cur"], sc["time_scan_end"])
fe = LioSamFrontEnd(LioSamParams(N_SCAN=64, Horizon_SCAN=2048))
fe.set_deskew(*tb[:4], sc["time_scan_cur"], tb[4])
fe.upload(sc["x"], sc["y"], sc["z"], sc["intensity"], sc["ring"], sc["time"])
for rep in range(5):
    fe.run()
buf = (C.c_ulonglong * (256 * 36 * 6))()
assert lib.slio_dbg_fe_stamps(buf) == 0
v = np.array(buf[:], dtype=np.int64).reshape(256, 36, 6)[:64]
live = v[:, :, 5] > 0
t0 = v[:, :, 0][live].min()
ph = np.diff(v, axis=2) / 100.0  # us
names = ["loads", "reach", "edges", "flats", "labels+out"]
for k, nm in enumerate(names):
    x = ph[:, :, k][live]
    print(f"{nm:10s} mean {x.mean():6.2f} p90 {np.quantile(x, .9):6.2f} max {x.max():6.2f} us")
st = (v[:, :, 0][live] - t0) / 100.0
en = (v[:, :, 5][live] - t0) / 100.0
print(f"start spread {st.max():.2f} us; end max {en.max():.2f} us; block total mean {(en - st).mean():.2f}")
lib.slio_dbg_ring_stamps.argtypes = [C.POINTER(C.c_ulonglong)]
rb = (C.c_ulonglong * (256 * 8))()
assert lib.slio_dbg_ring_stamps(rb) == 0
rv = np.array(rb[:], dtype=np.int64).reshape(256, 8)[:64]
if (rv[:, 4] == 0).all():  # presorted VoxelGrid order (ring_vsort): stamps 0-3 and 7
    rp = np.stack([rv[:, 1] - rv[:, 0], rv[:, 2] - rv[:, 1], rv[:, 3] - rv[:, 2], rv[:, 7] - rv[:, 3]], 1) / 100.0
    phases = ["hdr+chain", "labels+corners", "keep label<=0", "centroids"]
else:
    rp = np.diff(rv, axis=1) / 100.0
    phases = ["hdr+chain", "labels+corners", "surface scan", "bbox", "keys", "sort", "centroids"]
for k, nm in enumerate(phases):
    print(f"ring {nm:15s} mean {rp[:, k].mean():6.2f} max {rp[:, k].max():6.2f} us")
print(f"ring kernel: start spread {(rv[:, 0].max() - rv[:, 0].min()) / 100:.2f} us, "
      f"total mean {((rv[:, 7] - rv[:, 0]) / 100).mean():.2f} us")
lib.slio_dbg_vsort_stamps.argtypes = [C.POINTER(C.c_ulonglong)]
vb = (C.c_ulonglong * (256 * 4))()
assert lib.slio_dbg_vsort_stamps(vb) == 0
vv = np.array(vb[:], dtype=np.int64).reshape(256, 4)[:64]
ok = vv[:, 3] > 0
vp = np.diff(vv[ok], axis=1) / 100.0
narrow = "?"
print(f"vsort: keys {vp[:, 0].mean():.2f} sort {vp[:, 1].mean():.2f} out {vp[:, 2].mean():.2f} us; "
      f"total mean {((vv[ok, 3] - vv[ok, 0]) / 100).mean():.2f} max {((vv[ok, 3] - vv[ok, 0]) / 100).max():.2f}; "
      f"end (vs the sector blocks' first start) max {((vv[ok, 3] - t0) / 100).max():.2f} us")
fe.close()
