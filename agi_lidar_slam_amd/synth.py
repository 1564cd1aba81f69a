"""Seeded synthetic scenes, maps and scans for the IKF core.

Scene: ground plane z = 0 plus axis-aligned box buildings on a block grid.
Map: every surface sampled on a 0.5 m jittered grid (filter_size_map 0.5,
launch/mapping_avia.launch:13) with N(0, 1 cm) normal noise, float32, exactly
``n_map`` unique points.  Scan: ray-cast from a ground-truth pose with a
Livox-Avia-like rosette (70.4 deg FOV) or a VLP-16 pattern, N(0, 2 cm) range
noise, in LiDAR (body) frame.  The Avia scan keeps at most one return per
0.2 m voxel (a denser stand-in for feats_down_body after the 0.5 m VoxelGrid,
laserMapping.cpp:737-739: 100k voxel-unique 0.5 m returns are not visible
from one pose of this scene); the VLP-16 scan keeps every return.  Initial state =
ground truth boxplus (U(+-0.1 m)^3, U(+-0.5 deg)^3), extrinsic from
config/avia.yaml.  numpy's PCG64 makes every output platform-independent.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

AVIA_T_LI = np.array([0.04165, 0.02326, -0.0284])  # config/avia.yaml extrinsic_T
BLOCK = 60.0          # building block pitch (m)
MAP_RES = 0.5         # map sampling grid (m)
PTS_PER_BLOCK = 23200.0  # approx. surface samples per block (ground + building)


@dataclass
class Scene:
    half: float                       # ground covers [-half, half]^2
    boxes: np.ndarray                 # (B, 6) x0 y0 x1 y1 z0 z1


@dataclass
class Frame:
    """One synthetic scan with its ground truth."""
    body: np.ndarray                  # (N, 3) float32 LiDAR-frame points
    gt_rot: np.ndarray                # IMU rotation quaternion (w, x, y, z)
    gt_pos: np.ndarray
    init_rot: np.ndarray
    init_pos: np.ndarray
    t_li: np.ndarray = field(default_factory=lambda: AVIA_T_LI.copy())


def quat_from_rotvec(v: np.ndarray) -> np.ndarray:
    th = float(np.linalg.norm(v))
    if th < 1e-12:
        return np.array([1.0, 0.0, 0.0, 0.0])
    ax = v / th
    return np.concatenate([[np.cos(th / 2)], np.sin(th / 2) * ax])


def quat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([
        w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
        w1 * y2 + y1 * w2 + z1 * x2 - x1 * z2,
        w1 * z2 + z1 * w2 + x1 * y2 - y1 * x2,
    ])


def quat_matrix(q: np.ndarray) -> np.ndarray:
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def make_scene(seed: int, n_map: int) -> Scene:
    rng = np.random.default_rng(seed)
    nb = max(3, int(np.ceil(np.sqrt(n_map / PTS_PER_BLOCK))))
    if nb % 2 == 0:
        nb += 1
    half = nb * BLOCK / 2.0
    boxes = []
    for i in range(nb):
        for j in range(nb):
            cx = -half + (i + 0.5) * BLOCK
            cy = -half + (j + 0.5) * BLOCK
            w = rng.uniform(15.0, 40.0)
            d = rng.uniform(15.0, 40.0)
            h = rng.uniform(6.0, 35.0)
            # keep the street around the origin free for the sensor
            ox = rng.uniform(-(BLOCK - w) / 2 + 6.0, (BLOCK - w) / 2 - 6.0) if BLOCK - w > 12 else 0.0
            oy = rng.uniform(-(BLOCK - d) / 2 + 6.0, (BLOCK - d) / 2 - 6.0) if BLOCK - d > 12 else 0.0
            x0, y0 = cx + ox - w / 2, cy + oy - d / 2
            boxes.append([x0, y0, x0 + w, y0 + d, 0.0, h])
    return Scene(half=half, boxes=np.array(boxes, dtype=np.float64))


def _grid_samples(rng, u0, u1, v0, v1):
    """Jittered 0.5 m grid over a rectangle: returns (u, v) sample coords."""
    nu = max(1, int(np.floor((u1 - u0) / MAP_RES)))
    nv = max(1, int(np.floor((v1 - v0) / MAP_RES)))
    uu = u0 + (np.arange(nu) + 0.5) * ((u1 - u0) / nu)
    vv = v0 + (np.arange(nv) + 0.5) * ((v1 - v0) / nv)
    U, V = np.meshgrid(uu, vv, indexing="ij")
    U = U.ravel() + rng.uniform(-0.2, 0.2, U.size) * MAP_RES
    V = V.ravel() + rng.uniform(-0.2, 0.2, V.size) * MAP_RES
    return U, V


def sample_map(scene: Scene, seed: int, n_map: int) -> np.ndarray:
    """Exactly n_map unique float32 map points (N, 3)."""
    rng = np.random.default_rng(seed + 1)
    parts = []
    half = scene.half
    # ground, in strips to bound memory; drop samples under buildings
    strip = 60.0
    x = -half
    while x < half - 1e-9:
        U, V = _grid_samples(rng, x, min(x + strip, half), -half, half)
        inside = np.zeros(U.size, dtype=bool)
        for b in scene.boxes:
            if b[2] < x or b[0] > x + strip:
                continue
            inside |= (U >= b[0]) & (U <= b[2]) & (V >= b[1]) & (V <= b[3])
        U, V = U[~inside], V[~inside]
        parts.append(np.stack([U, V, rng.normal(0.0, 0.01, U.size)], 1))
        x += strip
    for b in scene.boxes:
        x0, y0, x1, y1, z0, z1 = b
        U, V = _grid_samples(rng, x0, x1, y0, y1)           # roof
        parts.append(np.stack([U, V, z1 + rng.normal(0.0, 0.01, U.size)], 1))
        for (a0, a1, c, axis) in ((x0, x1, y0, 1), (x0, x1, y1, 1), (y0, y1, x0, 0), (y0, y1, x1, 0)):
            U, V = _grid_samples(rng, a0, a1, z0, z1)
            W = c + rng.normal(0.0, 0.01, U.size)
            if axis == 1:
                parts.append(np.stack([U, W, V], 1))
            else:
                parts.append(np.stack([W, U, V], 1))
    pts = np.concatenate(parts).astype(np.float32)
    # unique float coordinates (ties in the kNN must not exist)
    v = np.ascontiguousarray(pts).view(np.dtype((np.void, 12))).ravel()
    _, first = np.unique(v, return_index=True)
    pts = pts[np.sort(first)]
    if pts.shape[0] < n_map:
        raise ValueError(f"scene too small: {pts.shape[0]} < {n_map}")
    keep = rng.choice(pts.shape[0], n_map, replace=False)
    return np.ascontiguousarray(pts[keep])


def _cast(scene: Scene, org: np.ndarray, dirs: np.ndarray, max_range: float) -> np.ndarray:
    """Distance along each unit ray to the first surface (inf if none)."""
    n = dirs.shape[0]
    t = np.full(n, np.inf)
    dz = dirs[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        tg = -org[2] / dz
    ok = (dz < 0) & (tg > 0)
    gx = org[0] + dirs[:, 0] * tg
    gy = org[1] + dirs[:, 1] * tg
    ok &= (np.abs(gx) <= scene.half) & (np.abs(gy) <= scene.half)  # ground exists only on the map
    t[ok] = tg[ok]
    B = scene.boxes
    # cull boxes beyond max_range of the origin
    cx = np.clip(org[0], B[:, 0], B[:, 2]) - org[0]
    cy = np.clip(org[1], B[:, 1], B[:, 3]) - org[1]
    B = B[np.hypot(cx, cy) <= max_range]
    lo = B[:, [0, 1, 4]]
    hi = B[:, [2, 3, 5]]
    for s in range(0, n, 8192):
        d = dirs[s:s + 8192]
        with np.errstate(divide="ignore", invalid="ignore"):
            inv = 1.0 / d
            t0 = (lo[None, :, :] - org[None, None, :]) * inv[:, None, :]
            t1 = (hi[None, :, :] - org[None, None, :]) * inv[:, None, :]
        tmin = np.nanmax(np.minimum(t0, t1), axis=2)
        tmax = np.nanmin(np.maximum(t0, t1), axis=2)
        hit = (tmax >= tmin) & (tmax > 0) & (tmin > 0)
        tb = np.where(hit, tmin, np.inf).min(axis=1)
        t[s:s + 8192] = np.minimum(t[s:s + 8192], tb)
    t[t > max_range] = np.inf
    return t


def _avia_dirs(k0: int, n: int) -> np.ndarray:
    """Rosette directions in the LiDAR frame (x forward), 70.4 deg FOV."""
    i = np.arange(k0, k0 + n, dtype=np.float64)
    phi = i * 0.0127
    rho = np.deg2rad(35.2) * np.abs(np.sin(2.618 * phi + 0.31 * np.floor(i / 7919.0)))
    az = rho * np.cos(phi)
    el = rho * np.sin(phi)
    return np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], 1)


def _vlp16_dirs(k0: int, n: int) -> np.ndarray:
    i = np.arange(k0, k0 + n)
    ring = i % 16
    rev = i // 16
    el = np.deg2rad(-15.0 + 2.0 * ring)
    az = (rev % 1250) * (2 * np.pi / 1250) + (rev // 1250) * 0.00113
    return np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], 1)


SENSOR_STREET = (BLOCK / 2, BLOCK / 2)  # a street crossing: buildings stay >= 6 m from it


def make_frame(scene: Scene, seed: int, n_scan: int, pattern: str = "avia",
               max_range: float = 300.0, voxel: float | None = None,
               sensor: str = "street") -> Frame:
    """voxel: one return per voxel of this edge (default 0.2 m for the Avia
    rosette; 0 = keep every return, default for the VLP-16 ring pattern).

    sensor: "street" puts the sensor near the street crossing at
    (BLOCK/2, BLOCK/2) +- 3 m, where no building can stand (make_scene keeps
    every building >= 6 m inside its block).  "origin" is the placement used
    before round 2, near (0, 0): the centre of the middle block, i.e. INSIDE
    a building for every scene size.  Rays do not hit the inside of their own
    box, so such a scan holds ground returns under the building's footprint,
    where the map has no samples (the 5th neighbour of ~9 % of the points of
    the 50M-point scene's scan lies 2.5-13.5 m away); kept as the hard case
    for scan points without map support."""
    if voxel is None:
        voxel = 0.2 if pattern == "avia" else 0.0
    rng = np.random.default_rng(seed + 2)
    yaw = rng.uniform(-np.pi, np.pi)
    if sensor == "street":
        # look along one of the two streets (+-18 deg), as a vehicle would:
        # facing a wall 6 m away the rosette would not find n_scan returns
        # that are voxel-unique at 0.2 m
        u = (yaw + np.pi) / (np.pi / 2)
        yaw = np.floor(u) * (np.pi / 2) + (u - np.floor(u) - 0.5) * 0.628
    gt_rot = quat_mul(quat_from_rotvec(np.array([0, 0, yaw])),
                      quat_from_rotvec(rng.uniform(-0.02, 0.02, 3)))
    gt_pos = np.array([rng.uniform(-3, 3), rng.uniform(-3, 3), 1.6])
    if sensor == "street":
        gt_pos[:2] += SENSOR_STREET
    elif sensor != "origin":
        raise ValueError(f"sensor must be 'street' or 'origin', not {sensor!r}")
    body = _render(scene, gt_rot, gt_pos, n_scan, pattern, max_range, voxel, rng)
    init_rot = quat_mul(gt_rot, quat_from_rotvec(rng.uniform(-1, 1, 3) * np.deg2rad(0.5)))
    init_pos = gt_pos + rng.uniform(-0.1, 0.1, 3)
    return Frame(body=np.ascontiguousarray(body), gt_rot=gt_rot, gt_pos=gt_pos,
                 init_rot=init_rot, init_pos=init_pos)


def _render(scene: Scene, gt_rot: np.ndarray, gt_pos: np.ndarray, n_scan: int, pattern: str,
            max_range: float, voxel: float, rng) -> np.ndarray:
    """n_scan LiDAR-frame returns of the scene seen from the IMU pose (gt_rot, gt_pos)."""
    R = quat_matrix(gt_rot)
    org = R @ AVIA_T_LI + gt_pos
    dir_fn = _avia_dirs if pattern == "avia" else _vlp16_dirs
    allp, allk, k0 = [], [], 0
    pw = None
    for _ in range(12):
        n = max(2 * n_scan, 65536)
        dl = dir_fn(k0, n)
        k0 += n
        dw = dl @ R.T
        t = _cast(scene, org, dw, max_range)
        ok = np.isfinite(t)
        tt = t[ok] + rng.normal(0.0, 0.02, ok.sum())
        p = org + dw[ok] * tt[:, None]
        allp.append(p)
        if voxel > 0:
            keys = np.floor(p / voxel).astype(np.int64)
            allk.append((keys[:, 0] * 73856093) ^ (keys[:, 1] * 19349663) ^ (keys[:, 2] * 83492791))
            kk = np.concatenate(allk)
            _, first = np.unique(kk, return_index=True)
        else:
            first = np.arange(sum(a.shape[0] for a in allp))
        if first.size >= n_scan:
            first = np.sort(first)[:n_scan]
            pw = np.concatenate(allp)[first]
            break
    if pw is None:
        raise ValueError(f"could not collect {n_scan} voxel-unique returns")
    body = ((pw - gt_pos) @ R - AVIA_T_LI).astype(np.float32)  # R_LI = I
    return body


def make_trajectory(seed: int, n_map: int, n_frames: int, n_scan: int, step: float = 0.5,
                    pattern: str = "avia", voxel: float | None = None) -> list:
    """Frames of a vehicle driving along the street y = BLOCK/2 (+x), `step`
    metres per scan, with a small yaw / roll wobble; init_* = ground truth (a
    mapping sequence carries its own state)."""
    if voxel is None:
        voxel = 0.2 if pattern == "avia" else 0.0
    scene = make_scene(seed, n_map)
    rng = np.random.default_rng(seed + 11)
    out = []
    for k in range(n_frames):
        gt_rot = quat_mul(quat_from_rotvec(np.array([0, 0, 0.05 * np.sin(0.3 * k)])),
                          quat_from_rotvec(rng.uniform(-0.01, 0.01, 3)))
        gt_pos = np.array([SENSOR_STREET[0] - 3.0 + step * k, SENSOR_STREET[1] + 0.3 * np.sin(0.2 * k), 1.6])
        body = _render(scene, gt_rot, gt_pos, n_scan, pattern, 300.0, voxel, rng)
        out.append(Frame(body=body, gt_rot=gt_rot, gt_pos=gt_pos, init_rot=gt_rot.copy(),
                         init_pos=gt_pos.copy()))
    return out


def make_problem(n_map: int, n_scan: int, seed: int = 20261015, pattern: str = "avia",
                 cache_dir: str | None = None, sensor: str = "street"):
    """(map_xyz float32 (M,3), Frame) for a config; cached as .npz if asked."""
    if cache_dir:
        os.makedirs(cache_dir, exist_ok=True)
        fn = os.path.join(cache_dir, f"slio2_{pattern}_{sensor}_{n_map}_{n_scan}_{seed}.npz")
        if os.path.exists(fn):
            z = np.load(fn)
            fr = Frame(body=z["body"], gt_rot=z["gt_rot"], gt_pos=z["gt_pos"],
                       init_rot=z["init_rot"], init_pos=z["init_pos"])
            return z["map"], fr
    scene = make_scene(seed, n_map)
    mp = sample_map(scene, seed, n_map)
    fr = make_frame(scene, seed, n_scan, pattern, sensor=sensor)
    if cache_dir:
        # several ranks may build the same problem at once: write a private
        # file and rename it into place, so no rank ever loads a partial one
        tmp = f"{fn}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            np.savez(f, map=mp, body=fr.body, gt_rot=fr.gt_rot, gt_pos=fr.gt_pos,
                     init_rot=fr.init_rot, init_pos=fr.init_pos)
        os.replace(tmp, fn)
    return mp, fr


def voxel_order(body: np.ndarray, leaf: float = 0.2) -> np.ndarray:
    """Permutation putting a scan in pcl::VoxelGrid output order: points sorted
    by voxel index idx = i + j * div_x + k * div_x * div_y over the cloud's
    bounding box (x fastest), the order in which laserMapping's
    downSizeFilterSurf emits feats_down_body (laserMapping.cpp:737-739).  The
    synthetic Avia scan is voxel-unique at `leaf`, so the order is total."""
    ijk = np.floor(body.astype(np.float64) / leaf).astype(np.int64)
    ijk -= ijk.min(axis=0)
    div = ijk.max(axis=0) + 1
    idx = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    return np.argsort(idx, kind="stable")


# ---------------------------------------------------------------- C3: Ouster
OUSTER_FOV_DEG = 16.6  # OS1-64: elevation -16.6 .. +16.6 deg


def make_ouster_scan(seed: int = 20261015, n_scan: int = 64, horizon: int = 2048,
                     yaw_rate: float = 0.5, dropout: float = 0.05, n_map_scene: int = 2_000_000,
                     time_scan_cur: float = 1000.0) -> dict:
    """One OS1-64-like sweep: n_scan x horizon returns in
    ring-major order (the PointCloud2 layout of the Ouster driver), per-point
    relative time from the column (t u32 ns -> t * 1e-9f, imageProjection.cpp
    :244-258), azimuth jitter of +-0.6 column so that cells collide and go
    empty, `dropout` zero returns, and a 200 Hz IMU stream with angular
    velocity (0, 0, yaw_rate) covering the sweep.  The sensor turns during the
    sweep, so each point is in the sensor frame of its own capture time."""
    scene = make_scene(seed, n_map_scene)
    rng = np.random.default_rng(seed + 3)
    yaw0 = rng.uniform(-np.pi, np.pi)
    org = np.array([rng.uniform(-3, 3), rng.uniform(-3, 3), 1.8])
    res = 2 * np.pi / horizon
    rows = np.repeat(np.arange(n_scan), horizon)
    cols = np.tile(np.arange(horizon), n_scan)
    el = np.deg2rad(-OUSTER_FOV_DEG + rows * (2 * OUSTER_FOV_DEG / (n_scan - 1)))
    az = (cols - horizon // 2 + rng.uniform(-0.6, 0.6, rows.size)) * res
    t_ns = np.round(cols * (1e8 / horizon)).astype(np.uint32)
    t_rel = t_ns.astype(np.float32) * np.float32(1e-9)
    dl = np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], 1)
    yaw = yaw0 + yaw_rate * t_rel.astype(np.float64)
    cy, sy = np.cos(yaw), np.sin(yaw)
    dw = np.stack([cy * dl[:, 0] - sy * dl[:, 1], sy * dl[:, 0] + cy * dl[:, 1], dl[:, 2]], 1)
    rng_m = _cast(scene, org, dw, 120.0)
    ok = np.isfinite(rng_m) & (rng.uniform(size=rows.size) >= dropout)
    r = np.where(ok, rng_m + rng.normal(0.0, 0.01, rows.size), 0.0)
    pts = (dl * r[:, None]).astype(np.float32)  # sensor frame at capture time
    intensity = rng.uniform(0.0, 255.0, rows.size).astype(np.float32)
    t_end = time_scan_cur + float(t_rel[-1])
    stamps = np.arange(time_scan_cur - 0.0475, t_end + 0.05, 0.005)
    gyro = np.tile([0.0, 0.0, yaw_rate], (stamps.size, 1)) + rng.normal(0, 1e-3, (stamps.size, 3))
    return dict(x=np.ascontiguousarray(pts[:, 0]), y=np.ascontiguousarray(pts[:, 1]),
                z=np.ascontiguousarray(pts[:, 2]), intensity=intensity,
                ring=rows.astype(np.uint16), time=t_rel, imu_stamps=stamps, imu_gyro=gyro,
                time_scan_cur=time_scan_cur, time_scan_end=t_end, n_scan=n_scan, horizon=horizon)


# ---------------------------------------------------------------- LeGO-LOAM: VLP-16 + IMU
def make_vlp16_sweep(seed: int = 20261015, horizon: int = 1800, yaw_rate: float = 0.3,
                     dropout: float = 0.03, n_map_scene: int = 2_000_000,
                     time_scan_cur: float = 500.0) -> dict:
    """One VLP-16 sweep in firing order (16 lasers per azimuth step, the
    velodyne_pointcloud layout LeGO-LOAM reads), no-return points dropped,
    sensor turning at yaw_rate about z; plus a 200 Hz IMU stream (orientation,
    linear acceleration, angular velocity) covering the sweep."""
    scene = make_scene(seed, n_map_scene)
    rng = np.random.default_rng(seed + 4)
    yaw0 = rng.uniform(-np.pi, np.pi)
    org = np.array([rng.uniform(-3, 3), rng.uniform(-3, 3), 1.7])
    cols = np.repeat(np.arange(horizon), 16)
    rings = np.tile(np.arange(16), horizon)
    t = cols * (0.1 / horizon)
    az = -(cols + rng.uniform(-0.3, 0.3, cols.size)) * (2 * np.pi / horizon) + np.pi  # clockwise
    el = np.deg2rad(-15.0 + 2.0 * rings + rng.normal(0, 0.02, cols.size))
    dl = np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], 1)
    yaw = yaw0 + yaw_rate * t
    cy, sy = np.cos(yaw), np.sin(yaw)
    dw = np.stack([cy * dl[:, 0] - sy * dl[:, 1], sy * dl[:, 0] + cy * dl[:, 1], dl[:, 2]], 1)
    r = _cast(scene, org, dw, 100.0)
    ok = np.isfinite(r) & (rng.uniform(size=cols.size) >= dropout)
    r = r + rng.normal(0.0, 0.01, cols.size)
    pts = (dl[ok] * r[ok, None]).astype(np.float32)
    stamps = np.arange(time_scan_cur - 0.2, time_scan_cur + 0.2, 0.005)
    ts = stamps - time_scan_cur
    imu = dict(time=stamps, roll=np.full(stamps.size, 0.01), pitch=np.full(stamps.size, -0.02),
               yaw=np.angle(np.exp(1j * (yaw0 + yaw_rate * ts))),
               acc=np.tile([0.1, 0.05, 9.81], (stamps.size, 1)) + rng.normal(0, 0.01, (stamps.size, 3)),
               gyro=np.tile([0.0, 0.0, yaw_rate], (stamps.size, 1)))
    return dict(x=np.ascontiguousarray(pts[:, 0]), y=np.ascontiguousarray(pts[:, 1]),
                z=np.ascontiguousarray(pts[:, 2]), time_scan_cur=time_scan_cur, imu=imu)


def s2m_lidar_pose(fr):
    """LIO-SAM's transformTobeMapped (roll, pitch, yaw, x, y, z) of a frame's
    ground-truth LiDAR pose, with its rotation matrix and translation."""
    R = quat_matrix(fr.gt_rot)
    t = fr.gt_pos + R @ AVIA_T_LI
    yaw = np.arctan2(R[1, 0], R[0, 0])
    pitch = np.arcsin(-R[2, 0])
    roll = np.arctan2(R[2, 1], R[2, 2])
    return np.array([roll, pitch, yaw, *t], np.float32), R, t


def make_s2m_problem(seed: int = 20261015, n_map: int = 200000, n_surf: int = 20000) -> dict:
    """A LIO-SAM scan-to-map problem (mapOptmization.cpp:1706-1740): the
    surf map sampled from the urban scene, a corner map along the buildings'
    vertical edges (0.1 m apart), the surf scan (an Avia-like frame) and the
    corner scan (edge points within 40 m of the sensor, in the LiDAR frame),
    and the ground-truth transformTobeMapped."""
    scene = make_scene(seed, n_map)
    surf_map = sample_map(scene, seed, n_map)
    rng = np.random.default_rng(4)
    lines = []
    for b in scene.boxes:
        for (cx, cy) in ((b[0], b[1]), (b[2], b[1]), (b[0], b[3]), (b[2], b[3])):
            z = np.arange(0.0, b[5], 0.1)
            lines.append(np.stack([cx + rng.normal(0, 0.005, z.size), cy + rng.normal(0, 0.005, z.size), z], 1))
    corner_map = np.concatenate(lines).astype(np.float32)
    fr = make_frame(scene, seed, n_surf, "avia")
    tf, R, t = s2m_lidar_pose(fr)
    near = np.linalg.norm(corner_map[:, :2] - t[:2], axis=1) < 40
    cw = corner_map[near][::3]
    cw = cw + rng.normal(0, 0.01, cw.shape)
    corner_scan = ((cw - t) @ R).astype(np.float32)
    return dict(surf_map=surf_map, corner_map=corner_map, surf_scan=fr.body, corner_scan=corner_scan, tf=tf)
