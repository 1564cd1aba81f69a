"""Batched replay (BASELINE config C5): R scan updates in
flight at once on one GPU against a shared map.

"Replicas only" across scans: every replica is its own ``slio_handle`` (own
non-blocking HIP stream, own mapped control block, own scan), all reading one
device map through ``slio_map_share`` (include/slio.h), and runs the whole
``update_iterated_dyn_share_modified`` (esekfom.hpp:270-346) with
``slio_ikf_update_device`` from its own host thread (ctypes drops the GIL for
the call), so the R updates overlap on the device.  No collective.

Every replica replays a DIFFERENT scan of the same scene (own seed: own pose,
own returns), as replaying a bag would.  ``verify()`` runs each replica alone
first and ``run()`` checks the concurrent results against those bit for bit.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import time

import numpy as np

from . import _lib as L
from . import synth


def replay_frames(map_points: int, scan_points: int, replicas: int, seed: int = 20261015,
                  cache_dir: str | None = None, first: int = 0):
    """The map and `replicas` distinct voxel-ordered scans of the same scene
    (scan r uses the r-th usable seed after `seed`; cached as npz)."""
    mp, _ = synth.make_problem(map_points, scan_points, pattern="avia", seed=seed, cache_dir=cache_dir)
    scene = None
    frames = []
    next_seed = seed
    for r in range(first + replicas):
        fn = os.path.join(cache_dir, f"replay2_{map_points}_{scan_points}_{r}.npz") if cache_dir else None
        if fn and os.path.exists(fn):
            z = np.load(fn)
            next_seed = int(z["seed"])
            fr = synth.Frame(body=z["body"], gt_rot=z["gt_rot"], gt_pos=z["gt_pos"],
                             init_rot=z["init_rot"], init_pos=z["init_pos"])
        else:
            if scene is None:
                scene = synth.make_scene(seed, map_points)
            while True:   # a pose facing a wall may not yield enough voxel-unique returns
                next_seed += 17
                try:
                    fr = synth.make_frame(scene, next_seed, scan_points, "avia")
                    break
                except ValueError:
                    continue
            if fn:
                os.makedirs(cache_dir, exist_ok=True)
                tmp = f"{fn}.{os.getpid()}.tmp.npz"
                np.savez(tmp, seed=next_seed, body=fr.body, gt_rot=fr.gt_rot, gt_pos=fr.gt_pos,
                         init_rot=fr.init_rot, init_pos=fr.init_pos)
                os.replace(tmp, fn)
        if r >= first:
            fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
            frames.append(fr)
    return mp, frames


class _Rep:
    def __init__(self, lib, h, fr, iters):
        self.lib, self.h, self.iters = lib, h, iters
        xs0 = L.SlioState()
        xs0.pos[:] = list(fr.init_pos)
        xs0.rot[:] = list(fr.init_rot)
        xs0.rli[:] = [1.0, 0.0, 0.0, 0.0]
        xs0.tli[:] = list(synth.AVIA_T_LI)
        xs0.grav[:] = [0.0, 0.0, -9.81]
        self.xs0 = xs0
        self.xs = L.SlioState()
        self.P0 = np.eye(24) * 1e-2
        self.P = np.empty_like(self.P0)
        self.stats = L.SlioIkfStats()
        self.err = None
        self.cb = L.ALLREDUCE_FN()

    def step(self):
        # every step restarts from the scan's own prior (the same work per step)
        C.memmove(C.addressof(self.xs), C.addressof(self.xs0), C.sizeof(self.xs))
        self.P[...] = self.P0
        rc = self.lib.slio_ikf_update_device(self.h, C.byref(self.xs), L.dptr(self.P), 0.001, self.iters, 0,
                                             L.SLIO_MODE_FIXED, self.cb, None, C.byref(self.stats))
        L.check(rc, "ikf")

    def result(self):
        return bytes(memoryview(self.xs)), self.P.copy()


class Replay:
    """R replicas on `device`, one map uploaded once and shared."""

    def __init__(self, mp, frames, device=0, iters=4, cell=0.0):
        self.lib = L.load()
        lib = self.lib
        self.handles = []
        for fr in frames:
            p = L.SlioParams()
            lib.slio_params_default(C.byref(p))
            p.device, p.max_points, p.rank, p.nranks = device, fr.body.shape[0], 0, 1
            p.grid_cell = cell
            h = C.c_void_p()
            L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
            self.handles.append(h)
        x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
        L.check(lib.slio_map_upload(self.handles[0], L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
        for h in self.handles[1:]:
            L.check(lib.slio_map_share(h, self.handles[0]), "share")
        for h, fr in zip(self.handles, frames):
            bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
            L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]), "scan")
        self.reps = [_Rep(lib, h, fr, iters) for h, fr in zip(self.handles, frames)]
        self.ref = None

    def cell(self) -> float:
        c = C.c_float()
        L.check(self.lib.slio_map_info(self.handles[0], None, C.byref(c), None), "map_info")
        return float(c.value)

    def verify(self):
        """Each replica alone, one after the other: the reference results."""
        self.ref = []
        for rep in self.reps:
            rep.step()
            self.ref.append(rep.result())

    def solo_rate(self, steps, warmup):
        rep = self.reps[0]
        for _ in range(warmup):
            rep.step()
        t0 = time.perf_counter()
        for _ in range(steps):
            rep.step()
        return steps * rep.iters / (time.perf_counter() - t0)

    def run(self, steps, warmup, before=None, after=None):
        """All replicas concurrently (one host thread each); `before` / `after`
        run on the calling thread right before / after the timed region (e.g.
        a cross-rank barrier).  Returns the timed seconds."""
        R = len(self.reps)
        go = threading.Barrier(R + 1)
        done = threading.Barrier(R + 1)

        def work(rep):
            try:
                for _ in range(warmup):
                    rep.step()
                go.wait()
                go.wait()
                for _ in range(steps):
                    rep.step()
                done.wait()
            except Exception as e:  # reported after the join
                rep.err = e
                for b in (go, done):
                    try:
                        b.abort()
                    except Exception:
                        pass

        th = [threading.Thread(target=work, args=(rep,)) for rep in self.reps]
        for t in th:
            t.start()
        el = 0.0
        try:
            go.wait()
            if before:
                before()
            t0 = time.perf_counter()
            go.wait()
            done.wait()
            el = time.perf_counter() - t0
            if after:
                el = after(el)
        except threading.BrokenBarrierError:
            pass
        for t in th:
            t.join()
        for rep in self.reps:
            if rep.err:
                raise rep.err
        return el

    def identical(self) -> bool:
        if self.ref is None:
            return False
        return all(rep.result()[0] == rx and np.array_equal(rep.P, rP)
                   for rep, (rx, rP) in zip(self.reps, self.ref))

    def close(self):
        for h in reversed(self.handles):
            self.lib.slio_destroy(h)
        self.handles = []
