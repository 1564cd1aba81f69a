"""CPU analysis of pass-0 refinement work (diagnostic, not a test).

For the C2 problem at its initial pose: which queries the 3x3x3 block does
not finish, and how many candidates the 5x5x5 refinement scans under
different bounds (the current one, and the ideal: cells within the true
5th distance).  Grid aligned to the map's minimum (the device pads it; the
statistics, not the exact cells, are what this is for)."""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agi_lidar_slam_amd import synth  # noqa: E402

H = 1.25
mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
Rl = synth.quat_matrix(np.array([1.0, 0, 0, 0]))
R = synth.quat_matrix(np.asarray(fr.init_rot))
q = ((fr.body[:, :3].astype(np.float64) @ Rl.T + synth.AVIA_T_LI) @ R.T + fr.init_pos).astype(np.float32)
o = mp.min(0) - 2 * H
cm = np.floor((mp - o) / H).astype(np.int64)
dims = cm.max(0) + 3
lin = (cm[:, 2] * dims[1] + cm[:, 1]) * dims[0] + cm[:, 0]
cnt = np.bincount(lin, minlength=int(np.prod(dims)))
tree = cKDTree(mp)
d, _ = tree.query(q, k=5)
d5 = d[:, 4].astype(np.float64) ** 2
cq = np.floor((q - o) / H).astype(np.int64)


def cube(c, r):
    return [(c[0] + a, c[1] + b, c[2] + e) for e in range(-r, r + 1) for b in range(-r, r + 1)
            for a in range(-r, r + 1)]


def cell_count(x, y, z):
    if min(x, y, z) < 0 or x >= dims[0] or y >= dims[1] or z >= dims[2]:
        return 0
    return int(cnt[(z * dims[1] + y) * dims[0] + x])


def gap2(p, c):
    lo = o + np.asarray(c) * H
    g = np.maximum(np.maximum(lo - p, p - (lo + H)), 0)
    return float((g * g).sum())


def bound(p, c, r):
    lo = o + (np.asarray(c) - r) * H
    hi = lo + (2 * r + 1) * H
    return float(min((p - lo).min(), (hi - p).min()))


rows = []
for i in range(q.shape[0]):
    c = cq[i]
    p = q[i].astype(np.float64)
    blk = sum(cell_count(*cc) for cc in cube(c, 1))
    b1 = bound(p, c, 1)
    rows.append((i, blk, b1))
rows = np.array(rows)
blk = rows[:, 1]
b1 = rows[:, 2]
# the block's 5th distance equals the true one when the true one is inside b1
done = (blk >= 5) & (d5 < b1 * b1 * 0.99999)
ref = ~done
print(f"queries {q.shape[0]}; block not done: {ref.sum()}  (block < 5 points: {(blk < 5).sum()})")
T_cur, T_ideal, starv = [], [], []
for i in np.nonzero(ref)[0]:
    c = cq[i]
    p = q[i].astype(np.float64)
    b2 = bound(p, c, 2)
    # current lim: block d5 if the block had 5 and it lies inside the cube, else INF
    # (block d5 >= true d5; approximated by the true d5 when the block had 5)
    lim = d5[i] if (blk[i] >= 5 and d5[i] < b2 * b2) else np.inf
    starv.append(not np.isfinite(lim))
    tc = ti = 0
    inner = set(cube(c, 1))
    for cc in cube(c, 2):
        if cc in inner:
            continue
        g = gap2(p, cc)
        n = cell_count(*cc)
        if g <= lim:
            tc += n
        if g <= d5[i]:
            ti += n
    T_cur.append(tc)
    T_ideal.append(ti)
T_cur = np.array(T_cur)
T_ideal = np.array(T_ideal)
starv = np.array(starv)
for name, m in (("all", np.ones_like(starv)), ("starved (lim=inf)", starv), ("lim=d5", ~starv)):
    if m.any():
        print(f"{name}: n={m.sum()} candidates now mean {T_cur[m].mean():.0f} p90 {np.quantile(T_cur[m], .9):.0f} "
              f"max {T_cur[m].max()}; within true d5: mean {T_ideal[m].mean():.0f} max {T_ideal[m].max()}")
print("true d5 (m) of starved: ", np.round(np.sqrt(d5[np.nonzero(ref)[0][starv]][:20]), 2))
