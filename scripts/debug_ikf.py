"""Device vs host IKF loop on the C1 problem: prints state / P / stats per maxit."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402
from agi_lidar_slam_amd.esekf import Esekf, KdTreeMap, StateIkfom  # noqa: E402

np.set_printoptions(precision=6, linewidth=160)
mp, fr = synth.make_problem(200000, 20000, pattern="vlp16")
st = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9),
                     [0, 0, -9.81]])
kd = KdTreeMap()
kd.Build(mp)
for mode in (1, 0):
    for maxit in (1, 2, 3):
        out = {}
        for dl in (False, True):
            kf = Esekf()
            kf.change_x(StateIkfom.from_array(st))
            kf.change_P(np.eye(24) * 1e-2)
            kf.update_iterated_dyn_share_modified(0.001, fr.body, kd, None, maxit, False,
                                                  mode=mode, device_loop=dl)
            s = kf.last_stats
            out[dl] = (kf.get_x().to_array(), kf.get_P().copy(),
                       (s.passes, s.searches, s.valid_passes, s.converged, s.last_m))
            kf.close()
        (xh, Ph, sh), (xd, Pd, sd) = out[False], out[True]
        print(f"mode {mode} maxit {maxit}: host stats {sh} dev stats {sd}")
        print("  host x", xh[:7])
        print("  dev  x", xd[:7])
        print("  |dx| max", np.abs(xh - xd).max(), " |dP| max", np.abs(Ph - Pd).max(),
              " P diag dev", np.diag(Pd)[:6])
kd.close()
