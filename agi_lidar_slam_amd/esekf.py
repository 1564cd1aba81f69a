"""Python mirror of the reference's filter interface on the MI355X path.

Names, argument meaning and error behaviour follow
``esekfom::esekf`` (src/S-FAST_LIO/include/esekfom.hpp:42-351),
``state_ikfom`` (use-ikfom.hpp:18-27) and the parts of ``KD_TREE`` the IKF
uses (Build, size; ikd_Tree.h:45-299).  Every numeric pass runs on the GPU
through libslio.so (include/slio.h); this module only marshals arguments.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L

G_M_S2 = 9.81          # common_lib.h:21
LASER_POINT_COV = 0.001  # laserMapping.cpp:29
NUM_MATCH_POINTS = 5   # common_lib.h:22


@dataclass
class StateIkfom:
    """state_ikfom (use-ikfom.hpp:18-27); rotations as unit quaternions (w, x, y, z)."""
    pos: np.ndarray = field(default_factory=lambda: np.zeros(3))
    rot: np.ndarray = field(default_factory=lambda: np.array([1.0, 0, 0, 0]))
    offset_R_L_I: np.ndarray = field(default_factory=lambda: np.array([1.0, 0, 0, 0]))
    offset_T_L_I: np.ndarray = field(default_factory=lambda: np.zeros(3))
    vel: np.ndarray = field(default_factory=lambda: np.zeros(3))
    bg: np.ndarray = field(default_factory=lambda: np.zeros(3))
    ba: np.ndarray = field(default_factory=lambda: np.zeros(3))
    grav: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, -G_M_S2]))

    def to_c(self) -> L.SlioState:
        s = L.SlioState()
        for name, arr in (("pos", self.pos), ("rot", self.rot), ("rli", self.offset_R_L_I),
                          ("tli", self.offset_T_L_I), ("vel", self.vel), ("bg", self.bg),
                          ("ba", self.ba), ("grav", self.grav)):
            getattr(s, name)[:] = [float(v) for v in arr]
        return s

    @staticmethod
    def from_c(s: L.SlioState) -> "StateIkfom":
        return StateIkfom(pos=np.array(s.pos[:]), rot=np.array(s.rot[:]),
                          offset_R_L_I=np.array(s.rli[:]), offset_T_L_I=np.array(s.tli[:]),
                          vel=np.array(s.vel[:]), bg=np.array(s.bg[:]), ba=np.array(s.ba[:]),
                          grav=np.array(s.grav[:]))

    def to_array(self) -> np.ndarray:
        """The 26 doubles of slio_state, in memory order."""
        return np.concatenate([self.pos, self.rot, self.offset_R_L_I, self.offset_T_L_I,
                               self.vel, self.bg, self.ba, self.grav]).astype(np.float64)

    @staticmethod
    def from_array(a: np.ndarray) -> "StateIkfom":
        a = np.asarray(a, dtype=np.float64)
        return StateIkfom(pos=a[0:3].copy(), rot=a[3:7].copy(), offset_R_L_I=a[7:11].copy(),
                          offset_T_L_I=a[11:14].copy(), vel=a[14:17].copy(), bg=a[17:20].copy(),
                          ba=a[20:23].copy(), grav=a[23:26].copy())


def _params(device: int, max_points: int, rank: int, nranks: int, grid_cell: float,
            plane_threshold: float, max_match_sqd: float) -> L.SlioParams:
    lib = L.load()
    p = L.SlioParams()
    L.check(lib.slio_params_default(C.byref(p)), "slio_params_default")
    p.device, p.max_points, p.rank, p.nranks = device, max_points, rank, nranks
    p.grid_cell, p.plane_threshold, p.max_match_sqd = grid_cell, plane_threshold, max_match_sqd
    return p


class _Handle:
    def __init__(self, params: L.SlioParams):
        self.lib = L.load()
        self.h = C.c_void_p()
        L.check(self.lib.slio_create(C.byref(self.h), C.byref(params)), "slio_create")
        self.params = params

    def close(self):
        if self.h:
            self.lib.slio_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class KdTreeMap(_Handle):
    """Stands where ``KD_TREE<PointType> ikdtree`` stands (static snapshot).

    ``Build`` mirrors KD_TREE::Build (ikd_Tree.cpp:355-367); neighbour indices
    reported by the filter refer to rows of the array passed to Build.
    """

    def __init__(self, device: int = 0, grid_cell: float = 0.0):  # 0: the library's auto edge
        super().__init__(_params(device, 1, 0, 1, grid_cell, 0.1, 5.0))
        self.points = np.zeros((0, 3), np.float32)
        # bumped by every Build: a filter bound to this map re-shares it (a
        # share holds the device map of the moment it was made)
        self.generation = 0

    def Build(self, points: np.ndarray) -> None:
        pts = np.ascontiguousarray(np.asarray(points, dtype=np.float32)[:, :3])
        x, y, z = (np.ascontiguousarray(pts[:, k]) for k in range(3))
        L.check(self.lib.slio_map_upload(self.h, L.fptr(x), L.fptr(y), L.fptr(z), pts.shape[0]),
                "KdTreeMap.Build")
        self.points = pts   # the Build snapshot (ids 0..n-1); flatten() gives the live map
        self.generation += 1

    def size(self) -> int:
        """KD_TREE::size (valid points; the device map after any changes)."""
        n = C.c_int64()
        L.check(self.lib.slio_map_info(self.h, None, None, C.byref(n)), "map_info")
        return int(n.value)

    def set_downsample_param(self, downsample_size: float) -> None:
        """KD_TREE::set_downsample_param (ikd_Tree.h:275), used by Add_Points."""
        self.downsample_size = float(downsample_size)

    def Add_Points(self, points: np.ndarray, downsample_on: bool) -> int:
        """KD_TREE::Add_Points (ikd_Tree.cpp:419-512) on the device map."""
        pts = np.ascontiguousarray(np.asarray(points, dtype=np.float32).reshape(-1, 3))
        x, y, z = (np.ascontiguousarray(pts[:, k]) for k in range(3))
        cnt = C.c_int64()
        L.check(self.lib.slio_map_add_points(self.h, L.fptr(x), L.fptr(y), L.fptr(z), pts.shape[0],
                                             int(downsample_on), getattr(self, "downsample_size", 0.2),
                                             C.byref(cnt)), "Add_Points")
        return int(cnt.value)

    def Delete_Point_Boxes(self, boxes: np.ndarray) -> int:
        """KD_TREE::Delete_Point_Boxes (ikd_Tree.cpp:559-579); boxes (k, 6) =
        vertex_min xyz, vertex_max xyz."""
        b = np.ascontiguousarray(np.asarray(boxes, dtype=np.float32).reshape(-1, 6))
        k = C.c_int64()
        L.check(self.lib.slio_map_delete_boxes(self.h, L.fptr(b.reshape(-1)), b.shape[0], C.byref(k)),
                "Delete_Point_Boxes")
        return int(k.value)

    def flatten(self):
        """(points (n, 3) f32, ids (n,) u32) of the valid map in ascending id."""
        n = C.c_int64()
        self.lib.slio_map_download(self.h, None, None, None, None, 0, C.byref(n))
        m = n.value
        x, y, z = (np.zeros(m, np.float32) for _ in range(3))
        ids = np.zeros(m, np.uint32)
        L.check(self.lib.slio_map_download(self.h, L.fptr(x), L.fptr(y), L.fptr(z),
                                           ids.ctypes.data_as(C.POINTER(C.c_uint32)), m, C.byref(n)),
                "flatten")
        return np.stack([x, y, z], 1), ids

    def grid_info(self):
        dims = (C.c_int32 * 3)()
        cell = C.c_float()
        n = C.c_int64()
        L.check(self.lib.slio_map_info(self.h, dims, C.byref(cell), C.byref(n)), "map_info")
        return tuple(dims), cell.value, n.value


@dataclass
class DynShareData:
    """dyn_share_datastruct (esekfom.hpp:32-40), reduced form."""
    valid: bool = True
    converge: bool = True
    HTH: np.ndarray | None = None   # 12x12
    HTh: np.ndarray | None = None   # 12
    m: int = 0


class Esekf(_Handle):
    """esekfom::esekf on the MI355X path."""

    def __init__(self, device: int = 0, max_points: int = 100000, rank: int = 0,
                 nranks: int = 1, plane_threshold: float = 0.1, max_match_sqd: float = 5.0):
        super().__init__(_params(device, max_points, rank, nranks, 1.0, plane_threshold,
                                 max_match_sqd))
        self.x_ = StateIkfom()
        self.P_ = np.eye(24)
        self._map_src = None
        self._map_gen = -1
        self._scan_ref = None
        self.last_stats = L.SlioIkfStats()

    # --- accessors (esekfom.hpp:50-56)
    def get_x(self) -> StateIkfom:
        return self.x_

    def get_P(self) -> np.ndarray:
        return self.P_

    def change_x(self, x: StateIkfom) -> None:
        self.x_ = x

    def change_P(self, P: np.ndarray) -> None:
        self.P_ = np.array(P, dtype=np.float64).reshape(24, 24)

    # --- plumbing
    def downsample_scan(self, feats_undistort: np.ndarray, filter_size_surf: float) -> int:
        """downSizeFilterSurf.filter (laserMapping.cpp:737-739) on the device:
        the downsampled scan stays in HBM as this filter's feats_down_body
        (pass feats_down_body=None to the update to use it).  Returns
        feats_down_size."""
        pts = np.ascontiguousarray(np.asarray(feats_undistort, dtype=np.float32)[:, :3])
        x, y, z = (np.ascontiguousarray(pts[:, k]) for k in range(3))
        n = C.c_int64()
        L.check(self.lib.slio_scan_upload_voxel(self.h, L.fptr(x), L.fptr(y), L.fptr(z), pts.shape[0],
                                                float(filter_size_surf), C.byref(n)), "downsample_scan")
        self._scan_ref = None
        self._n_scan = int(n.value)
        return self._n_scan

    def feats_down_body(self) -> np.ndarray:
        """The handle's current scan (feats_down_body) as an (n, 3) array."""
        b, e = C.c_int64(), C.c_int64()
        L.check(self.lib.slio_shard_range(self.h, C.byref(b), C.byref(e)), "shard_range")
        n = getattr(self, "_n_scan", 0)
        x, y, z = (np.zeros(n, np.float32) for _ in range(3))
        L.check(self.lib.slio_scan_download(self.h, L.fptr(x), L.fptr(y), L.fptr(z)), "scan_download")
        return np.stack([x, y, z], 1)

    def _bind(self, feats_down_body: np.ndarray | None, ikdtree: KdTreeMap) -> int:
        if self._map_src is not ikdtree or self._map_gen != ikdtree.generation:
            L.check(self.lib.slio_map_share(self.h, ikdtree.h), "map_share")
            self._map_src = ikdtree
            self._map_gen = ikdtree.generation
        if feats_down_body is None:   # the device scan of downsample_scan
            return getattr(self, "_n_scan", 0)
        pts = np.ascontiguousarray(np.asarray(feats_down_body, dtype=np.float32)[:, :3])
        x, y, z = (np.ascontiguousarray(pts[:, k]) for k in range(3))
        L.check(self.lib.slio_scan_upload(self.h, L.fptr(x), L.fptr(y), L.fptr(z), pts.shape[0]),
                "scan_upload")
        self._scan_ref = feats_down_body
        self._n_scan = int(pts.shape[0])
        return pts.shape[0]

    def boxplus(self, x: StateIkfom, f: np.ndarray) -> StateIkfom:
        out = L.SlioState()
        f = np.ascontiguousarray(f, dtype=np.float64)
        xc = x.to_c()
        L.check(self.lib.slio_state_boxplus(C.byref(xc), L.dptr(f), C.byref(out)), "boxplus")
        return StateIkfom.from_c(out)

    def boxminus(self, x1: StateIkfom, x2: StateIkfom) -> np.ndarray:
        d = np.zeros(24)
        a, b = x1.to_c(), x2.to_c()
        L.check(self.lib.slio_state_boxminus(C.byref(a), C.byref(b), L.dptr(d)), "boxminus")
        return d

    def h_share_model(self, ekfom_data: DynShareData, feats_down_body: np.ndarray,
                      ikdtree: KdTreeMap, Nearest_Points: dict | None,
                      extrinsic_est: bool) -> None:
        """One measurement pass (esekfom.hpp:106-227); search iff ekfom_data.converge."""
        if (feats_down_body is not self._scan_ref or self._map_src is not ikdtree
                or self._map_gen != ikdtree.generation):
            # (feats_down_body None: the device scan of downsample_scan)
            self._bind(feats_down_body, ikdtree)
        pose = L.SlioPose()
        pose.rot[:] = list(self.x_.rot)
        pose.pos[:] = list(self.x_.pos)
        pose.rli[:] = list(self.x_.offset_R_L_I)
        pose.tli[:] = list(self.x_.offset_T_L_I)
        HTH = np.zeros(78)
        HTh = np.zeros(12)
        m = C.c_int64()
        L.check(self.lib.slio_iterate(self.h, C.byref(pose), int(ekfom_data.converge),
                                      int(extrinsic_est), L.dptr(HTH), L.dptr(HTh), C.byref(m)),
                "h_share_model")
        full = np.zeros((12, 12))
        full[np.triu_indices(12)] = HTH
        full = full + np.triu(full, 1).T
        ekfom_data.HTH, ekfom_data.HTh, ekfom_data.m = full, HTh, int(m.value)
        ekfom_data.valid = m.value >= 1
        if Nearest_Points is not None:
            Nearest_Points.update(self.nearest_points())

    def map_incremental(self, ikdtree: "KdTreeMap", filter_size_map_min: float = 0.5,
                        flg_EKF_inited: bool = True) -> np.ndarray:
        """map_incremental (laserMapping.cpp:382-433) on the device: the scan of
        the last update, at the current state, against its Nearest_Points.
        Returns (|PointToAdd|, |PointNoNeedDownsample|, Add_Points counter)."""
        if self._map_src is not ikdtree or self._map_gen != ikdtree.generation:
            raise ValueError("map_incremental: the last update ran on another map")
        counts = np.zeros(3, np.int64)
        xc = self.x_.to_c()
        L.check(self.lib.slio_map_incremental(self.h, C.byref(xc), float(filter_size_map_min),
                                              int(bool(flg_EKF_inited)), L.i64ptr(counts)),
                "map_incremental")
        return counts

    def nearest_points(self) -> dict:
        b, e = C.c_int64(), C.c_int64()
        L.check(self.lib.slio_shard_range(self.h, C.byref(b), C.byref(e)), "shard_range")
        n = e.value - b.value
        idx = np.zeros((n, 5), np.int32)
        sqd = np.zeros((n, 5), np.float32)
        sel = np.zeros(n, np.uint8)
        L.check(self.lib.slio_get_neighbors(self.h, L.iptr(idx), L.fptr(sqd), L.u8ptr(sel)),
                "get_neighbors")
        return {"index": idx, "sq_dist": sqd, "selected": sel.astype(bool), "begin": b.value}

    def planes(self) -> np.ndarray:
        b, e = C.c_int64(), C.c_int64()
        self.lib.slio_shard_range(self.h, C.byref(b), C.byref(e))
        out = np.zeros((e.value - b.value, 4), np.float32)
        L.check(self.lib.slio_get_planes(self.h, L.fptr(out)), "get_planes")
        return out

    def update_iterated_dyn_share_modified(self, R: float, feats_down_body: np.ndarray,
                                           ikdtree: KdTreeMap, Nearest_Points: dict | None,
                                           maximum_iter: int, extrinsic_est: bool,
                                           mode: int = L.SLIO_MODE_REFERENCE,
                                           reduce=None, device_loop: bool = True) -> None:
        """esekfom.hpp:270-346.  device_loop=True: slio_ikf_update_device (state,
        covariance and control flow resident in HBM, one host sync per update);
        False: slio_ikf_update (host C++ 24x24 algebra after every pass)."""
        self._bind(feats_down_body, ikdtree)
        xc = self.x_.to_c()
        P = np.ascontiguousarray(self.P_, dtype=np.float64).copy()
        cb = reduce if reduce is not None else L.ALLREDUCE_FN()
        st = L.SlioIkfStats()
        fn = self.lib.slio_ikf_update_device if device_loop else self.lib.slio_ikf_update
        L.check(fn(self.h, C.byref(xc), L.dptr(P), float(R), int(maximum_iter),
                   int(extrinsic_est), int(mode), cb, None, C.byref(st)),
                "update_iterated_dyn_share_modified")
        self.x_ = StateIkfom.from_c(xc)
        self.P_ = P.reshape(24, 24)
        self.last_stats = st
        if Nearest_Points is not None:
            Nearest_Points.update(self.nearest_points())
