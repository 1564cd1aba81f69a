"""A synthetic UndistortPcl case shared by the CPU and GPU IMU tests."""
import numpy as np


def make_case(seed=0, first_late=False, n=30000):
    rng = np.random.default_rng(seed)
    beg, end = 100.0, 100.1
    ts = np.arange(beg - 0.004, end + 0.006, 0.005)
    w = np.array([0.1, -0.2, 0.8]) + rng.normal(0, 0.01, (ts.size, 3))
    a = np.array([0.3, 0.1, 1.02]) + rng.normal(0, 0.02, (ts.size, 3))
    imu = np.concatenate([ts[:, None], a, w], 1)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pts = (d * rng.uniform(2, 80, (n, 1))).astype(np.float32)
    t = rng.uniform(0, 100, n).astype(np.float32)
    t[:50] = 0.0                                   # points at the scan start: not moved
    t[50:300] = np.round(t[50:300])                # time ties
    if first_late:
        t = np.maximum(t, 12.0).astype(np.float32)  # first point past the 2nd IMU pose
    state = np.concatenate([[1.0, -2.0, 0.5], [0.99, 0.02, -0.03, 0.1], [1, 0, 0, 0],
                            [0.04165, 0.02326, -0.0284], [1.5, 0.2, 0.0], [0.001, -0.002, 0.0005],
                            [0.01, 0.02, -0.01], [0.0, 0.0, -9.81]])
    state[3:7] /= np.linalg.norm(state[3:7])
    P = np.eye(24) * 1e-3
    cov12 = np.array([0.1] * 3 + [0.1] * 3 + [1e-4] * 3 + [1e-4] * 3)
    return dict(imu=imu, beg=beg, end=end, last_end=beg - 0.002, mean_acc_norm=float(np.linalg.norm([0.3, 0.1, 1.02])),
                cov12=cov12, acc_s_last=np.array([0.1, 0.0, 0.05]), angvel_last=np.array([0.1, -0.2, 0.8]),
                state=state, P=P, pts=pts, t=t)
