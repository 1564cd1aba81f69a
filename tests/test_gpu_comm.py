"""GPU tests of the in-library multi-GPU path (include/slio.h).

The reference updates on one CPU process (laserMapping.cpp:772-774); the
drop-in shards the scan over ranks and all-reduces each pass's 8 x 91 fp64
super rows inside the library (esekfom.hpp:306-319 summed over the shards):

* slio_create_group / slio_group_ikf_update (one process, one handle per
  rank).  On this one-GPU box the ranks share the device, so the group takes
  the in-device reduce backend (SLIO_GROUP_DEVICE: k_group_reduce on rank 0's
  stream between every rank's pass and every rank's filter step, ordered by
  HIP events) -- the same enqueue -> all-reduce -> k_ikf_solve -> bitwise
  agreement sequence as with RCCL.  N = 1, 2, 4, 8 ranks at C2 size, both
  control flows and extrinsic estimation: x, P and the stats bit for bit
  equal to the plain single-rank update, and within the north_star tolerance
  of the oracle.  A group of one rank takes the RCCL backend.
* slio_comm_unique_id / slio_comm_init (one process per GPU, torchrun):
  one rank, reduce == NULL, bitwise equal to the single-rank update.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_gpu_parity import L, mk, rot_err, state_of, upload_map, upload_scan  # noqa: E402,F401
from test_gpu_runtime import C2_CELL, TOL_POS, TOL_ROT, c2, slio_state, state_array  # noqa: E402,F401

pytestmark = pytest.mark.gpu


def single_update(L, mp, fr, st, maxit=4, mode=None, ext=0):
    lib = L.load()
    mode = L.SLIO_MODE_FIXED if mode is None else mode
    h = mk(L, cell=C2_CELL)
    try:
        upload_map(L, h, mp)
        assert upload_scan(L, h, fr.body) == 0
        xs = slio_state(st)
        P = np.eye(24) * 1e-2
        stt = L.SlioIkfStats()
        L.check(lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, maxit, ext, mode,
                                           L.ALLREDUCE_FN(), None, C.byref(stt)), "single")
        return state_array(xs), P, (stt.passes, stt.searches, stt.valid_passes, stt.last_m)
    finally:
        lib.slio_destroy(h)


def group_update(L, mp, fr, st, devices, maxit=4, mode=None, ext=0, kinds=None, updates=1):
    """One group of len(devices) ranks: rank 0 takes the map, ranks on the
    same device share it, every rank takes the whole scan; `updates`
    back-to-back group updates from the same prior (the last one returned)."""
    lib = L.load()
    mode = L.SLIO_MODE_FIXED if mode is None else mode
    n = len(devices)
    p = L.SlioParams()
    lib.slio_params_default(C.byref(p))
    p.max_points, p.grid_cell = fr.body.shape[0], C2_CELL
    hs = (C.c_void_p * n)()
    dv = (C.c_int32 * n)(*devices)
    rc = lib.slio_create_group(hs, n, dv, C.byref(p))
    if rc:
        return rc, lib.slio_last_error().decode(), None
    try:
        if kinds is not None:
            kinds.extend(lib.slio_group_reduce_kind(hs[r]) for r in range(n))
        upload_map(L, hs[0], mp)
        for r in range(1, n):
            if devices[r] == devices[0]:
                L.check(lib.slio_map_share(hs[r], hs[0]), "share")
            else:
                upload_map(L, hs[r], mp)
        for r in range(n):
            assert upload_scan(L, hs[r], fr.body) == 0
        for _ in range(updates):
            xs = slio_state(st)
            P = np.eye(24) * 1e-2
            stt = L.SlioIkfStats()
            rc = lib.slio_group_ikf_update(hs, n, C.byref(xs), L.dptr(P), 0.001, maxit, ext, mode,
                                           C.byref(stt))
            if rc:
                return rc, lib.slio_last_error().decode(), None
        return 0, "", (state_array(xs), P, (stt.passes, stt.searches, stt.valid_passes, stt.last_m))
    finally:
        for r in range(n):
            lib.slio_destroy(hs[r])


@pytest.mark.parametrize("mode", [0, 1])
def test_group_one_rank_bitwise(L, oracle_mod, c2, mode):
    mp, fr, T = c2
    st = state_of(fr)
    x1, P1, s1 = single_update(L, mp, fr, st, mode=mode)
    rc, msg, out = group_update(L, mp, fr, st, [0], mode=mode)
    assert rc == 0, msg
    xg, Pg, sg = out
    np.testing.assert_array_equal(xg, x1)
    np.testing.assert_array_equal(Pg, P1)
    assert sg == s1
    s_ref, *_ = oracle_mod.ikf_update(T, fr.body, st, np.eye(24) * 1e-2, maximum_iter=4, mode=mode,
                                      reference_gain=0)
    assert np.abs(xg[0:3] - s_ref[0:3]).max() < TOL_POS
    assert rot_err(xg[3:7], s_ref[3:7]) < TOL_ROT


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("mode,ext", [(1, 0), (0, 0), (0, 1)])
def test_group_ranks_one_device_bitwise(L, oracle_mod, c2, mode, ext, fused, monkeypatch):
    """C4's in-library sequence at N = 2, 4, 8 ranks on this one GPU (the
    in-device reduce backend): bitwise equal to one rank, in the FIXED and the
    REFERENCE control flow, with and without extrinsic estimation; the group
    is updated twice (its counters, gates and events are reused).  fused: one
    launch per rank per pass (the ranks' super rows into the group's buffer,
    the filter step in the rank that arrives last) plus a gate launch between
    passes; else (SLIO_NO_FUSE=1) search + super-sum launches, events,
    k_group_reduce and a filter-step launch per rank."""
    if not fused:
        monkeypatch.setenv("SLIO_NO_FUSE", "1")
    mp, fr, T = c2
    st = state_of(fr)
    x1, P1, s1 = single_update(L, mp, fr, st, mode=mode, ext=ext)
    s_ref, *_ = oracle_mod.ikf_update(T, fr.body, st, np.eye(24) * 1e-2, maximum_iter=4, mode=mode,
                                      reference_gain=0, extrinsic=bool(ext))
    assert np.abs(x1[0:3] - s_ref[0:3]).max() < TOL_POS
    assert rot_err(x1[3:7], s_ref[3:7]) < TOL_ROT
    for n in (2, 4, 8):
        kinds = []
        rc, msg, out = group_update(L, mp, fr, st, [0] * n, mode=mode, ext=ext, kinds=kinds, updates=2)
        assert rc == 0, msg
        assert kinds == [L.SLIO_GROUP_DEVICE] * n
        xg, Pg, sg = out
        np.testing.assert_array_equal(xg, x1)
        np.testing.assert_array_equal(Pg, P1)
        assert sg == s1


def test_group_rccl_refused_on_shared_device(L, c2, monkeypatch):
    """SLIO_GROUP_REDUCE=rccl cannot put two ranks on one device: a clear
    error, no handles left behind."""
    mp, fr, _ = c2
    monkeypatch.setenv("SLIO_GROUP_REDUCE", "rccl")
    rc, msg, _ = group_update(L, mp, fr, state_of(fr), [0, 0])
    assert rc == -1 and "one device per rank" in msg


def test_comm_init_one_rank_bitwise(L, c2):
    """slio_comm_unique_id + slio_comm_init (the torchrun form) with one rank:
    the update all-reduces in the library (reduce == NULL)."""
    mp, fr, _ = c2
    st = state_of(fr)
    x1, P1, s1 = single_update(L, mp, fr, st)
    lib = L.load()
    h = mk(L, cell=C2_CELL)
    try:
        uid = (C.c_uint8 * L.SLIO_COMM_ID_BYTES)()
        L.check(lib.slio_comm_unique_id(uid), "unique id")
        L.check(lib.slio_comm_init(h, uid), "comm init")
        upload_map(L, h, mp)
        assert upload_scan(L, h, fr.body) == 0
        xs = slio_state(st)
        P = np.eye(24) * 1e-2
        stt = L.SlioIkfStats()
        L.check(lib.slio_ikf_update_device(h, C.byref(xs), L.dptr(P), 0.001, 4, 0, L.SLIO_MODE_FIXED,
                                           L.ALLREDUCE_FN(), None, C.byref(stt)), "comm update")
        np.testing.assert_array_equal(state_array(xs), x1)
        np.testing.assert_array_equal(P, P1)
        assert (stt.passes, stt.searches, stt.valid_passes, stt.last_m) == s1
    finally:
        lib.slio_destroy(h)


@pytest.mark.parametrize("n", [2, 8])
def test_group_gate_timeout_reported_and_recovers(L, c2, n):
    """A gate between fused group passes that gives up (forced here through
    slio_debug_wait_limit(rank 0, 1): every gate gives up at once, so the
    ranks' passes run without waiting for the group's filter step and their
    arrivals on the group counter mix passes) is reported as its own error,
    SLIO_ETIMEOUT, never as a result; the group's and every rank's arrival
    counters are reset, so the next update (normal wait) is bitwise equal to
    one rank alone."""
    mp, fr, _ = c2
    st = state_of(fr)
    x1, P1, s1 = single_update(L, mp, fr, st)
    lib = L.load()
    p = L.SlioParams()
    lib.slio_params_default(C.byref(p))
    p.max_points, p.grid_cell = fr.body.shape[0], C2_CELL
    hs = (C.c_void_p * n)()
    dv = (C.c_int32 * n)(*([0] * n))
    L.check(lib.slio_create_group(hs, n, dv, C.byref(p)), "group")
    try:
        upload_map(L, hs[0], mp)
        for r in range(1, n):
            L.check(lib.slio_map_share(hs[r], hs[0]), "share")
        for r in range(n):
            assert upload_scan(L, hs[r], fr.body) == 0

        def update():
            xs = slio_state(st)
            P = np.eye(24) * 1e-2
            stt = L.SlioIkfStats()
            rc = lib.slio_group_ikf_update(hs, n, C.byref(xs), L.dptr(P), 0.001, 4, 0, L.SLIO_MODE_FIXED,
                                           C.byref(stt))
            return rc, state_array(xs), P, (stt.passes, stt.searches, stt.valid_passes, stt.last_m)

        L.check(lib.slio_debug_wait_limit(hs[0], 1), "wait limit")
        for _ in range(2):
            rc, *_ = update()
            assert rc == L.SLIO_ETIMEOUT, (rc, lib.slio_last_error().decode())
            assert "gave up" in lib.slio_last_error().decode()
        L.check(lib.slio_debug_wait_limit(hs[0], 0), "wait limit")
        for _ in range(2):
            rc, xg, Pg, sg = update()
            assert rc == 0, lib.slio_last_error().decode()
            np.testing.assert_array_equal(xg, x1)
            np.testing.assert_array_equal(Pg, P1)
            assert sg == s1
    finally:
        for r in range(n):
            lib.slio_destroy(hs[r])
