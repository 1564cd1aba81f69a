"""Generate the committed golden vectors under tests/golden/.

Independent of both the product and the oracle:
  * knn_golden.npz   — exact 5-NN by scipy.spatial.cKDTree (float64 query,
    k = 8), re-ranked by the reference's float32 distance
    ((dx*dx + dy*dy) + dz*dz, ikd_Tree.cpp:1539-1544) and kept only where the
    5th and 6th float32 distances differ (tie-free);
  * plane_golden.npz — planes of those neighbour sets by numpy float64 least
    squares (A n = -1, common_lib.h:102-134), with the 0.1 m acceptance flag
    kept only where no residual lies within 1e-3 of the threshold.
Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from agi_lidar_slam_amd import synth  # noqa: E402


def f32_sqd(q, p):
    d = q.astype(np.float32)[:, None, :] - p.astype(np.float32)
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


def main():
    mp, fr = synth.make_problem(20000, 3000, seed=7, pattern="avia")
    rng = np.random.default_rng(11)
    R = synth.quat_matrix(fr.gt_rot)
    q = (fr.body.astype(np.float64) + synth.AVIA_T_LI) @ R.T + fr.gt_pos
    extra = np.concatenate([
        rng.uniform(mp.min(0) - 20, mp.max(0) + 20, (200, 3)),   # anywhere, incl. outside the bbox
        mp[rng.choice(mp.shape[0], 100)] + rng.normal(0, 0.3, (100, 3)),
        np.array([[1e3, 1e3, 50.0], [-1e3, 0, 0], [0, 0, 300.0]]),  # far outside the grid
    ])
    q = np.concatenate([q, extra]).astype(np.float32)
    tree = cKDTree(mp.astype(np.float64))
    _, ii = tree.query(q.astype(np.float64), 8)
    d32 = f32_sqd(q, mp[ii])
    order = np.lexsort((ii, d32), axis=1)
    ii = np.take_along_axis(ii, order, 1)
    d32 = np.take_along_axis(d32, order, 1)
    keep = d32[:, 5] > d32[:, 4]
    q, idx, sqd = q[keep], ii[keep, :5].astype(np.int32), d32[keep, :5]
    np.savez_compressed(os.path.join(HERE, "knn_golden.npz"), map=mp, query=q, idx=idx, sqd=sqd)

    # planes of near-surface neighbour sets
    near = sqd[:, 4] < 5.0
    nb = mp[idx[near]].astype(np.float64)
    planes, flags, nbs = [], [], []
    for k in range(nb.shape[0]):
        A = nb[k]
        n, *_ = np.linalg.lstsq(A, -np.ones(5), rcond=None)
        nn = np.linalg.norm(n)
        pl = np.concatenate([n / nn, [1.0 / nn]])
        res = np.abs(A @ pl[:3] + pl[3])
        if np.any(np.abs(res - 0.1) < 1e-3):
            continue
        planes.append(pl)
        flags.append(bool(np.all(res <= 0.1)))
        nbs.append(mp[idx[near]][k])
    np.savez_compressed(os.path.join(HERE, "plane_golden.npz"), nb=np.array(nbs, np.float32),
                        plane=np.array(planes), ok=np.array(flags))
    print("knn", q.shape[0], "plane", len(planes), "accepted", int(np.sum(flags)))


if __name__ == "__main__":
    main()
