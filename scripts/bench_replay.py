#!/usr/bin/env python3
"""C5 batched replay on one GPU: R scan updates in flight at once on a shared map.

SURVEY.md §8(e) C5: "replicas only" across scans — every replica is its own
`slio_handle` (own non-blocking HIP stream, own mapped control block, own scan),
all reading one device map through `slio_map_share` (include/slio.h). Each
replica runs `slio_ikf_update_device` (the whole `update_iterated_dyn_share_modified`,
esekfom.hpp:270-346) from its own host thread; ctypes drops the GIL for the call,
so the R updates overlap on the device. No collective: replicas are independent.

Every replica runs a DIFFERENT scan of the same scene (own seed: own pose,
own returns), as replaying a bag would; a replica's map reads therefore do
not coincide with the others' in L2 / MALL.

value = IKF iterations of all replicas / wall time of the timed region. Every
replica's result is checked bitwise against its own scan run alone first, so
concurrency cannot change results.

  python scripts/bench_replay.py --replicas 4 --steps 50
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=4)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--map-points", type=int, default=10_000_000)
    ap.add_argument("--scan-points", type=int, default=100_000)
    ap.add_argument("--cell", type=float, default=0.0)  # auto: 1.25 m on the 50M map, 1.0 m on 10M
    ap.add_argument("--cache-dir", default=os.environ.get("SLIO_CACHE", "/tmp/slio_cache"))
    args = ap.parse_args()

    from agi_lidar_slam_amd import _lib as L, synth

    lib = L.load()
    R = args.replicas
    seed = 20261015
    t0 = time.time()
    mp, _ = synth.make_problem(args.map_points, args.scan_points, pattern="avia", seed=seed,
                               cache_dir=args.cache_dir)
    scene = synth.make_scene(seed, args.map_points)
    frames = []
    next_seed = seed
    for r in range(R):
        fn = os.path.join(args.cache_dir, f"replay2_{args.map_points}_{args.scan_points}_{r}.npz")
        if os.path.exists(fn):
            z = np.load(fn)
            next_seed = int(z["seed"])
            fr = synth.Frame(body=z["body"], gt_rot=z["gt_rot"], gt_pos=z["gt_pos"],
                             init_rot=z["init_rot"], init_pos=z["init_pos"])
        else:
            while True:   # a pose facing a wall may not yield enough voxel-unique returns
                next_seed += 17
                try:
                    fr = synth.make_frame(scene, next_seed, args.scan_points, "avia")
                    break
                except ValueError:
                    continue
            os.makedirs(args.cache_dir, exist_ok=True)
            np.savez(fn, seed=next_seed, body=fr.body, gt_rot=fr.gt_rot, gt_pos=fr.gt_pos, init_rot=fr.init_rot,
                     init_pos=fr.init_pos)
        fr.body = np.ascontiguousarray(fr.body[synth.voxel_order(fr.body)])
        frames.append(fr)
    print(f"[replay] map {mp.shape[0]} + {R} scans in {time.time() - t0:.1f}s", file=sys.stderr)

    handles = []
    for r in range(R):
        p = L.SlioParams()
        lib.slio_params_default(C.byref(p))
        p.device, p.max_points, p.rank, p.nranks = 0, args.scan_points, 0, 1
        p.grid_cell = args.cell
        h = C.c_void_p()
        L.check(lib.slio_create(C.byref(h), C.byref(p)), "create")
        handles.append(h)
    x, y, z = (np.ascontiguousarray(mp[:, k]) for k in range(3))
    L.check(lib.slio_map_upload(handles[0], L.fptr(x), L.fptr(y), L.fptr(z), mp.shape[0]), "map")
    for h in handles[1:]:
        L.check(lib.slio_map_share(h, handles[0]), "share")
    for h, fr in zip(handles, frames):
        bx, by, bz = (np.ascontiguousarray(fr.body[:, k]) for k in range(3))
        L.check(lib.slio_scan_upload(h, L.fptr(bx), L.fptr(by), L.fptr(bz), fr.body.shape[0]),
                "scan")

    P0 = np.eye(24) * 1e-2

    def prior(fr):
        xs0 = L.SlioState()
        xs0.pos[:] = list(fr.init_pos)
        xs0.rot[:] = list(fr.init_rot)
        xs0.rli[:] = [1.0, 0.0, 0.0, 0.0]
        xs0.tli[:] = list(synth.AVIA_T_LI)
        xs0.grav[:] = [0.0, 0.0, -9.81]
        return xs0
    reduce_cb = L.ALLREDUCE_FN()

    class Rep:
        def __init__(self, h, fr):
            self.h = h
            self.xs0 = prior(fr)
            self.xs = L.SlioState()
            self.P = np.empty_like(P0)
            self.stats = L.SlioIkfStats()
            self.err = None

        def step(self):
            C.memmove(C.addressof(self.xs), C.addressof(self.xs0), C.sizeof(self.xs))
            self.P[...] = P0
            rc = lib.slio_ikf_update_device(self.h, C.byref(self.xs), L.dptr(self.P), 0.001,
                                            args.iters, 0, L.SLIO_MODE_FIXED, reduce_cb, None,
                                            C.byref(self.stats))
            L.check(rc, "ikf")

    reps = [Rep(h, fr) for h, fr in zip(handles, frames)]
    # reference results: every replica alone, one after the other
    ref = []
    for rep in reps:
        rep.step()
        ref.append((bytes(memoryview(rep.xs)), rep.P.copy()))
    # single-replica rate (same harness) for the comparison line
    for _ in range(args.warmup):
        reps[0].step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        reps[0].step()
    single = args.steps * args.iters / (time.perf_counter() - t0)

    go = threading.Barrier(R + 1)

    def run(rep):
        try:
            for _ in range(args.warmup):
                rep.step()
            go.wait()
            go.wait()
            for _ in range(args.steps):
                rep.step()
        except Exception as e:  # reported after the join
            rep.err = e
            try:
                go.abort()
            except Exception:
                pass

    th = [threading.Thread(target=run, args=(rep,)) for rep in reps]
    for t in th:
        t.start()
    try:
        go.wait()
        t0 = time.perf_counter()
        go.wait()
    except threading.BrokenBarrierError:
        t0 = time.perf_counter()   # a replica failed: join, then report its error
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    for rep in reps:
        if rep.err:
            raise rep.err
    same = all(bytes(memoryview(rep.xs)) == rx and np.array_equal(rep.P, rP)
               for rep, (rx, rP) in zip(reps, ref))
    for h in reversed(handles):
        lib.slio_destroy(h)
    total = R * args.steps * args.iters / el
    print(json.dumps({
        "metric": "IKF iterations/sec, batched replay (C5), distinct 100k-pt scans vs shared map",
        "value": total, "unit": "IKF iterations/s", "replicas": R, "steps": args.steps,
        "map_points": args.map_points, "scan_points": args.scan_points,
        "single_replica_value": single, "speedup_vs_single": total / single,
        "results_identical_to_single": bool(same),
    }))
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
