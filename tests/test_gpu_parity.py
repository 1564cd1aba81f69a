"""GPU parity tests: the HIP path through the C-ABI vs the CPU oracle.

Bar (BASELINE.json north_star): bit-exact on kNN indices and
squared distances, selection flags, planes and residuals; H^T H / H^T h to
fp64 summation-order tolerance; filter state within 1e-4 m / 1e-5 rad (the
tests use 1e-6 m / 1e-7 rad).  Run on a MI355X:  pytest -m gpu
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL_POS = 1e-6   # m   (north_star bar 1e-4 m)
TOL_ROT = 1e-7   # rad (north_star bar 1e-5 rad)


@pytest.fixture(scope="module")
def L():
    from agi_lidar_slam_amd import build, _lib
    build.build()
    return _lib


def mk(L, n_max=100000, rank=0, nranks=1, cell=0.75, max_cells=0, radius=None, lpq=0, far=None):
    lib = L.load()
    p = L.SlioParams()
    lib.slio_params_default(C.byref(p))
    p.max_points, p.rank, p.nranks, p.grid_cell = n_max, rank, nranks, cell
    if radius is not None:
        p.search_radius = radius
    p.lanes_per_query = lpq
    if far is not None:
        p.far_query_margin = far
    if max_cells:
        p.max_grid_cells = max_cells
    h = C.c_void_p()
    L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
    return h


def upload_map(L, h, pts):
    pts = np.ascontiguousarray(pts, np.float32)
    x, y, z = (np.ascontiguousarray(pts[:, k]) for k in range(3))
    L.check(L.load().slio_map_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), pts.shape[0]), "map")


def upload_scan(L, h, pts):
    pts = np.ascontiguousarray(pts, np.float32)
    x, y, z = (np.ascontiguousarray(pts[:, k]) for k in range(3))
    return L.load().slio_scan_upload(h, L.fptr(x), L.fptr(y), L.fptr(z), pts.shape[0])


def pose_of(L, st):
    p = L.SlioPose()
    p.pos[:] = list(st[0:3])
    p.rot[:] = list(st[3:7])
    p.rli[:] = list(st[7:11])
    p.tli[:] = list(st[11:14])
    return p


IDENT = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0] + [0] * 9 + [0, 0, -9.81], float)


def iterate(L, h, st, search, ext=False):
    HTH = np.zeros(78)
    HTh = np.zeros(12)
    m = C.c_int64()
    pose = pose_of(L, st)
    L.check(L.load().slio_iterate(h, C.byref(pose), int(search), int(ext), L.dptr(HTH),
                                  L.dptr(HTh), C.byref(m)), "iterate")
    return np.concatenate([HTH, HTh, [m.value]])


def results(L, h, n):
    lib = L.load()
    idx = np.zeros((n, 5), np.int32)
    sqd = np.zeros((n, 5), np.float32)
    sel = np.zeros(n, np.uint8)
    pl = np.zeros((n, 4), np.float32)
    rs = np.zeros(n, np.float32)
    L.check(lib.slio_get_neighbors(h, L.iptr(idx), L.fptr(sqd), L.u8ptr(sel)), "nbrs")
    L.check(lib.slio_get_planes(h, L.fptr(pl)), "planes")
    L.check(lib.slio_get_residuals(h, L.fptr(rs)), "resid")
    return idx, sqd, sel, pl, rs


def state_of(fr, pos=None, rot=None):
    from agi_lidar_slam_amd import synth
    return np.concatenate([fr.init_pos if pos is None else pos,
                           fr.init_rot if rot is None else rot, [1, 0, 0, 0], synth.AVIA_T_LI,
                           np.zeros(9), [0, 0, -9.81]])


@pytest.fixture(scope="module")
def c1(oracle_mod):
    from agi_lidar_slam_amd import synth
    out = {}
    for pat in ("vlp16", "avia"):
        mp, fr = synth.make_problem(200000, 20000, pattern=pat)
        out[pat] = (mp, fr, oracle_mod.Tree(mp))
    return out


def assert_sums_close(got, ref):
    assert int(got[90]) == int(ref[90])
    scale = np.abs(ref[:90]).max() + 1e-30
    np.testing.assert_allclose(got[:90], ref[:90], rtol=1e-9, atol=1e-11 * scale)


# ------------------------------------------------------------------ kNN
def test_knn_golden_bitexact(L):
    z = np.load(os.path.join(GOLD, "knn_golden.npz"))
    h = mk(L, far=0.0)   # exact everywhere: the golden set has far-away queries
    try:
        upload_map(L, h, z["map"])
        assert upload_scan(L, h, z["query"]) == 0
        iterate(L, h, IDENT, True)   # identity pose: world query == input point
        idx, sqd, *_ = results(L, h, z["query"].shape[0])
        np.testing.assert_array_equal(idx, z["idx"])
        np.testing.assert_array_equal(sqd, z["sqd"])
    finally:
        L.load().slio_destroy(h)


@pytest.mark.parametrize("cell,max_cells,radius,lpq", [
    (0.37, 0, None, 0), (1.0, 0, None, 0), (2.5, 0, None, 0), (1.0, 4096, None, 0),
    (0.75, 0, 0.0, 0), (0.75, 0, 0.3, 0), (0.75, 0, 1.49, 0), (1.25, 0, 0.0, 2),
    (0.75, 0, 1.0, 1), (0.75, 0, 1.0, 4), (0.75, 0, 1.0, 8)])
def test_knn_grid_geometry_invariant(L, oracle_mod, c1, cell, max_cells, radius, lpq):
    """Exactness must not depend on the cell edge, the cell-budget fallback,
    the first-sphere radius or the lanes per query."""
    mp, fr, T = c1["avia"]
    st = state_of(fr)
    q = oracle_mod.body_to_world(st, fr.body)
    ridx, rsqd = T.knn(q, 5)
    h = mk(L, cell=cell, max_cells=max_cells, radius=radius, lpq=lpq)
    try:
        upload_map(L, h, mp)
        upload_scan(L, h, fr.body)
        iterate(L, h, st, True)
        idx, sqd, *_ = results(L, h, q.shape[0])
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_array_equal(sqd, rsqd)
    finally:
        L.load().slio_destroy(h)


@pytest.mark.parametrize("cell,lpq", [(0.75, 0), (1.25, 0), (1.25, 1), (1.0, 4)])
def test_knn_nine_run_path(L, oracle_mod, c1, monkeypatch, cell, lpq):
    """Without the block rows (SLIO_NO_BLOCK_ROWS, or a map too large for
    them) the 3x3x3 block is scanned as 9 runs of the cell-sorted map: the
    same candidates and keys, so the same bit-exact result."""
    monkeypatch.setenv("SLIO_NO_BLOCK_ROWS", "1")
    mp, fr, T = c1["avia"]
    st = state_of(fr)
    q = oracle_mod.body_to_world(st, fr.body)
    ridx, rsqd = T.knn(q, 5)
    h = mk(L, cell=cell, lpq=lpq)
    try:
        upload_map(L, h, mp)
        upload_scan(L, h, fr.body)
        iterate(L, h, st, True)
        idx, sqd, *_ = results(L, h, q.shape[0])
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_array_equal(sqd, rsqd)
    finally:
        L.load().slio_destroy(h)


# ------------------------------------------------------------------ repeated search
@pytest.mark.parametrize("shift", [[0.03, -0.02, 0.01], [0.3, 0.2, -0.1], [2.0, -1.5, 0.4]])
def test_repeated_search_bitexact(L, oracle_mod, c1, shift):
    """A second search of the same scan after a pose change (what every IKF
    iteration does) is bit-exact for small and large pose changes."""
    mp, fr, T = c1["avia"]
    st = state_of(fr)
    h = mk(L, cell=1.25)
    try:
        upload_map(L, h, mp)
        upload_scan(L, h, fr.body)
        iterate(L, h, st, True)
        st2 = st.copy()
        st2[0:3] += shift
        iterate(L, h, st2, True)
        q = oracle_mod.body_to_world(st2, fr.body)
        ridx, rsqd = T.knn(q, 5)
        idx, sqd, *_ = results(L, h, q.shape[0])
        np.testing.assert_array_equal(sqd, rsqd)
        np.testing.assert_array_equal(idx, ridx)
    finally:
        L.load().slio_destroy(h)


def test_neighbors_outlive_scan_and_map_changes(L, oracle_mod, c1):
    """Nearest_Points ids and pointSearchSqDis are derived from the search
    pass's neighbour positions when first read; they must still be the last
    SEARCH pass's (not a later reuse pass's pose) after the handle's scan or
    map has been replaced."""
    mp, fr, T = c1["avia"]
    st = state_of(fr)
    n = fr.body.shape[0]
    h = mk(L, cell=1.25)
    try:
        upload_map(L, h, mp)
        upload_scan(L, h, fr.body)
        iterate(L, h, st, True)
        st2 = st.copy()
        st2[0:3] += [0.4, -0.3, 0.1]
        iterate(L, h, st2, False)          # reuse pass: neighbours unchanged
        ridx, rsqd = T.knn(oracle_mod.body_to_world(st, fr.body), 5)
        upload_scan(L, h, fr.body[::-1])    # new scan of the same size
        idx, sqd, *_ = results(L, h, n)
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_array_equal(sqd, rsqd)
        iterate(L, h, st2, True)            # search the new scan, then replace the map
        ridx2, rsqd2 = T.knn(oracle_mod.body_to_world(st2, fr.body[::-1]), 5)
        upload_map(L, h, mp[: mp.shape[0] // 2])
        idx, sqd, *_ = results(L, h, n)
        np.testing.assert_array_equal(idx, ridx2)
        np.testing.assert_array_equal(sqd, rsqd2)
    finally:
        L.load().slio_destroy(h)


# ------------------------------------------------------------------ passes
@pytest.mark.parametrize("pat", ["vlp16", "avia"])
@pytest.mark.parametrize("ext", [False, True])
def test_search_and_reuse_pass_vs_oracle(L, oracle_mod, c1, pat, ext):
    mp, fr, T = c1[pat]
    n = fr.body.shape[0]
    st = state_of(fr)
    h = mk(L)
    try:
        upload_map(L, h, mp)
        upload_scan(L, h, fr.body)
        got = iterate(L, h, st, True, ext)
        ps = oracle_mod.PassState(n)
        ref = oracle_mod.h_pass(T, st, fr.body, ps, True, extrinsic=ext)
        idx, sqd, sel, pl, rs = results(L, h, n)
        np.testing.assert_array_equal(idx, ps.idx)
        np.testing.assert_array_equal(sqd, ps.sqd)
        np.testing.assert_array_equal(sel, ps.sel)
        np.testing.assert_array_equal(pl, ps.plane)
        np.testing.assert_array_equal(rs, ps.resid)
        assert_sums_close(got, ref)
        # non-search pass at a moved pose reuses neighbours/planes/selection
        st2 = st.copy()
        st2[0:3] += [0.03, -0.02, 0.01]
        got2 = iterate(L, h, st2, False, ext)
        ref2 = oracle_mod.h_pass(T, st2, fr.body, ps, False, extrinsic=ext)
        idx, sqd, sel, pl, rs = results(L, h, n)
        np.testing.assert_array_equal(sel, ps.sel)
        np.testing.assert_array_equal(rs, ps.resid)
        assert_sums_close(got2, ref2)
    finally:
        L.load().slio_destroy(h)


# ------------------------------------------------------------------ full IKF
def rot_err(q1, q2):
    return 2 * np.arccos(min(1.0, abs(float(np.dot(q1, q2)) / np.linalg.norm(q1) / np.linalg.norm(q2))))


@pytest.mark.parametrize("pat,maxit,mode,device_loop", [
    ("vlp16", 3, 0, True), ("avia", 4, 0, True), ("avia", 4, 1, True),
    ("vlp16", 3, 0, False), ("avia", 4, 1, False)])
def test_ikf_update_vs_oracle(L, oracle_mod, c1, pat, maxit, mode, device_loop):
    from agi_lidar_slam_amd.esekf import Esekf, KdTreeMap, StateIkfom
    mp, fr, T = c1[pat]
    st = state_of(fr)
    P0 = np.eye(24) * 1e-2
    s_ref, P_ref, stats, idx_ref, sqd_ref, sel_ref = oracle_mod.ikf_update(
        T, fr.body, st, P0, maximum_iter=maxit, mode=mode, reference_gain=0)
    kd = KdTreeMap()
    kd.Build(mp)
    kf = Esekf()
    kf.change_x(StateIkfom.from_array(st))
    kf.change_P(P0)
    nearest = {}
    kf.update_iterated_dyn_share_modified(0.001, fr.body, kd, nearest, maxit, False, mode=mode,
                                          device_loop=device_loop)
    x = kf.get_x().to_array()
    assert np.abs(x[0:3] - s_ref[0:3]).max() < TOL_POS
    assert rot_err(x[3:7], s_ref[3:7]) < TOL_ROT
    st_ = kf.last_stats
    assert (st_.passes, st_.searches, st_.valid_passes) == tuple(stats[:3])
    assert st_.last_m == stats[4]
    # after several passes the fp64 states differ in the last bits (fp64 sums
    # are ordered differently), so the last search ran on queries that may
    # differ by an ulp: neighbours agree, distances to float rounding.
    # (Bit-exactness at identical queries is asserted by the pass tests.)
    assert (nearest["index"] == idx_ref).all(axis=1).mean() > 0.999
    np.testing.assert_allclose(nearest["sq_dist"], sqd_ref, rtol=1e-4, atol=1e-6)
    assert (nearest["selected"] == sel_ref.astype(bool)).mean() > 0.999
    np.testing.assert_allclose(kf.get_P(), P_ref, atol=1e-8 * np.abs(P_ref).max())
    kf.close()
    kd.close()


# ------------------------------------------------------------------ edges
@pytest.mark.parametrize("far", [None, 100.0])
def test_edge_cases(L, far):
    """default far_query_margin 0: exact everywhere (ikd-Tree semantics);
    100 m: the query ~1.4e6 m outside the map gets no neighbours."""
    lib = L.load()
    h = mk(L, n_max=1000, far=far)
    try:
        # reuse before any search -> ESTATE; iterate before map -> ESTATE
        assert upload_scan(L, h, np.zeros((4, 3), np.float32)) == 0
        pose = pose_of(L, IDENT)
        assert lib.slio_iterate_async(h, C.byref(pose), 1, 0, None) == -5
        # tiny map: fewer than 5 points -> idx -1, never selected
        upload_map(L, h, np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32))
        q = np.array([[0.1, 0.1, 0], [5, 5, 5], [np.nan, 0, 0], [1e6, -1e6, 3]], np.float32)
        assert upload_scan(L, h, q) == 0
        assert lib.slio_iterate_async(h, C.byref(pose), 0, 0, None) == -5
        s = iterate(L, h, IDENT, True)
        assert s[90] == 0
        idx, sqd, sel, pl, rs = results(L, h, 4)
        near = [0, 1, 3] if far is None else [0, 1]
        assert (idx[near, :3] >= 0).all() and (idx[:, 3:] == -1).all()
        assert (idx[2] == -1).all() and not sel.any()
        if far is not None:
            assert (idx[3] == -1).all()
        assert list(idx[0, :3]) == [0, 1, 2]
        # capacity
        assert upload_scan(L, h, np.zeros((1001, 3), np.float32)) == -4
        # empty scan: m = 0 (dyn_share.valid = false)
        assert upload_scan(L, h, np.zeros((0, 3), np.float32)) == 0
        assert iterate(L, h, IDENT, True)[90] == 0
        # empty map
        upload_map(L, h, np.zeros((0, 3), np.float32))
        assert upload_scan(L, h, q[:2]) == 0
        assert iterate(L, h, IDENT, True)[90] == 0
    finally:
        lib.slio_destroy(h)


def test_sharded_handles_bitwise_equal(L, c1):
    """nranks = 1, 2, 4, 8 handles (all on this GPU) give identical sums, and
    tests/tree_model.py rebuilds every rank's super rows from its chunk
    partials bit for bit (the model the gloo tests use)."""
    lib = L.load()
    mp, fr, _ = c1["avia"]
    st = state_of(fr)
    base = mk(L)
    upload_map(L, base, mp)
    upload_scan(L, base, fr.body)
    pose = pose_of(L, st)
    ref = np.zeros(8 * 91)
    L.check(lib.slio_iterate_async(base, C.byref(pose), 1, 0, None), "it")
    L.check(lib.slio_super_download(base, L.dptr(ref)), "dl")
    import tree_model as TM
    lib.slio_dbg_chunk_partials.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
    nch = C.c_int64()

    def partials(h):
        out = np.zeros((TM.num_chunks(fr.body.shape[0]), 91))
        L.check(lib.slio_dbg_chunk_partials(h, out.ctypes.data, out.size, C.byref(nch)), "partials")
        return out
    # the test model of the tree (tests/tree_model.py, used by the gloo
    # tests) rebuilds the device's super rows from its chunk partials
    part_all = partials(base)
    np.testing.assert_array_equal(TM.super_rows(part_all).reshape(-1), ref)
    try:
        for nr in (2, 4, 8):
            acc = np.zeros(8 * 91)
            for r in range(nr):
                h = mk(L, rank=r, nranks=nr)
                L.check(lib.slio_map_share(h, base), "share")
                upload_scan(L, h, fr.body)
                part = np.zeros(8 * 91)
                L.check(lib.slio_iterate_async(h, C.byref(pose), 1, 0, None), "it")
                L.check(lib.slio_super_download(h, L.dptr(part)), "dl")
                b, e = C.c_int64(), C.c_int64()
                lib.slio_shard_range(h, C.byref(b), C.byref(e))
                assert (b.value, e.value) == TM.shard_range(fr.body.shape[0], r, nr)
                np.testing.assert_array_equal(TM.super_rows(partials(h), r, nr).reshape(-1), part)
                acc = acc + part   # exact: each slot has one non-zero contributor
                lib.slio_destroy(h)
            np.testing.assert_array_equal(acc, ref)
    finally:
        lib.slio_destroy(base)


def test_full_size_c2_properties(L, oracle_mod):
    """BASELINE config C2 (100k scan vs 10M map): exact kNN on a sample and
    size-independent properties of the whole pass."""
    from agi_lidar_slam_amd import synth
    mp, fr = synth.make_problem(10_000_000, 100_000, pattern="avia", cache_dir="/tmp/slio_cache")
    st = state_of(fr)
    h = mk(L)
    try:
        upload_map(L, h, mp)
        upload_scan(L, h, fr.body)
        s = iterate(L, h, st, True)
        idx, sqd, sel, pl, rs = results(L, h, fr.body.shape[0])
        assert (np.diff(sqd, axis=1) >= 0).all() and (idx >= 0).all()
        assert int(s[90]) == int(sel.sum()) and sel.mean() > 0.5
        rng = np.random.default_rng(0)
        pick = rng.choice(fr.body.shape[0], 4000, replace=False)
        q = oracle_mod.body_to_world(st, fr.body)[pick]
        T = oracle_mod.Tree(mp)
        ridx, rsqd = T.knn(q, 5)
        np.testing.assert_array_equal(idx[pick], ridx)
        np.testing.assert_array_equal(sqd[pick], rsqd)
        # the pass is deterministic (fixed reduction tree)
        s2 = iterate(L, h, st, True)
        np.testing.assert_array_equal(s, s2)
    finally:
        L.load().slio_destroy(h)


@pytest.mark.parametrize("mode,ext", [(0, False), (1, False), (0, True)])
def test_device_loop_matches_host_loop(L, c1, mode, ext):
    """slio_ikf_update_device (filter step on device) vs slio_ikf_update (host):
    the same information-form algebra in the same order; the device takes
    1/sqrt from v_rsq_f64 + Newton and OCML sin/cos/atan, so single ulps
    differ.  P = (I - K H) P cancels in well-observed directions and the
    weakly observed extrinsic block amplifies single-ulp differences, so P is
    held to 5e-8 of max |P| (measured: 1.7e-8 with extrinsic_est)."""
    from agi_lidar_slam_amd.esekf import Esekf, KdTreeMap, StateIkfom
    mp, fr, _ = c1["avia"]
    st = state_of(fr)
    kd = KdTreeMap()
    kd.Build(mp)
    out = []
    for dev in (False, True):
        kf = Esekf()
        kf.change_x(StateIkfom.from_array(st))
        kf.change_P(np.eye(24) * 1e-2)
        kf.update_iterated_dyn_share_modified(0.001, fr.body, kd, None, 4, ext, mode=mode,
                                              device_loop=dev)
        s = kf.last_stats
        out.append((kf.get_x().to_array(), kf.get_P().copy(),
                    (s.passes, s.searches, s.valid_passes, s.converged, s.last_m)))
        kf.close()
    (x0, P0, s0), (x1, P1, s1) = out
    assert s0 == s1
    np.testing.assert_allclose(x1, x0, rtol=0, atol=1e-9)
    np.testing.assert_allclose(P1, P0, rtol=0, atol=5e-8 * np.abs(P0).max())
    kd.close()


@pytest.mark.gpu
def test_batched_replay_concurrent_bitwise(L, c1):
    """C5 batched replay: 4 handles share one map (slio_map_share),
    each on its own stream, running slio_ikf_update_device from 4 host threads at
    once; every replica's x and P equal the update run alone, bit for bit."""
    import threading
    lib = L.load()
    mp, fr, _ = c1["avia"]
    st = state_of(fr)
    xs0 = L.SlioState()
    xs0.pos[:] = list(st[0:3])
    xs0.rot[:] = list(st[3:7])
    xs0.rli[:] = list(st[7:11])
    xs0.tli[:] = list(st[11:14])
    xs0.vel[:] = list(st[14:17])
    xs0.bg[:] = list(st[17:20])
    xs0.ba[:] = list(st[20:23])
    xs0.grav[:] = list(st[23:26])
    cb = L.ALLREDUCE_FN()
    hs = [mk(L) for _ in range(4)]
    try:
        upload_map(L, hs[0], mp)
        for h in hs[1:]:
            L.check(lib.slio_map_share(h, hs[0]), "share")
        for h in hs:
            upload_scan(L, h, fr.body)

        def run(h, out, reps):
            for _ in range(reps):
                xs = L.SlioState()
                C.memmove(C.addressof(xs), C.addressof(xs0), C.sizeof(xs))
                P = np.eye(24) * 1e-2
                stt = L.SlioIkfStats()
                rc = lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, 4, 0,
                                                L.SLIO_MODE_FIXED, cb, None, C.byref(stt))
                out.append((rc, bytes(memoryview(xs)), P.copy()))

        ref = []
        run(hs[0], ref, 1)
        assert ref[0][0] == 0, L.load().slio_last_error()
        outs = [[] for _ in hs]
        th = [threading.Thread(target=run, args=(h, o, 3)) for h, o in zip(hs, outs)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for o in outs:
            assert len(o) == 3
            for rc, xb, P in o:
                assert rc == 0
                assert xb == ref[0][1]
                np.testing.assert_array_equal(P, ref[0][2])
    finally:
        for h in reversed(hs):
            lib.slio_destroy(h)


def test_auto_cell_edge(L):
    """grid_cell 0 (the default): 1.0 m, or 1.25 m when the 1.0 m grid would
    exceed 2^27 cells (cell edge)."""
    lib = L.load()
    rng = np.random.default_rng(7)
    for extent, want in ((np.array([200.0, 200.0, 30.0]), 1.0),
                         (np.array([600.0, 600.0, 400.0]), 1.25)):
        pts = (rng.random((5000, 3)) * extent).astype(np.float32)
        h = mk(L, cell=0.0)
        try:
            upload_map(L, h, pts)
            cell = C.c_float()
            L.check(lib.slio_map_info(h, None, C.byref(cell), None), "info")
            assert cell.value == want
        finally:
            lib.slio_destroy(h)
