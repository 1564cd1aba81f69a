"""World-size-2 gloo test of the N>1 reduction path on CPU.

Each rank computes the super-chunk sums of its own shard of the per-point
rows (oracle rows stand in for the device rows), zeros elsewhere; a SUM
all-reduce must reproduce the single-rank tree bit for bit, which is what
makes 1/2/4/8-GPU runs identical (agi_lidar_slam_amd/shard.py)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _rows(n=5000, seed=1):
    from oracle import oracle as O
    from agi_lidar_slam_amd import synth
    mpts, fr = synth.make_problem(50000, n, seed=seed, pattern="avia")
    T = O.Tree(mpts)
    st = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9),
                         [0, 0, -9.81]])
    ps = O.PassState(n)
    rows = np.zeros((n, 14))
    O.h_pass(T, st, fr.body, ps, True, rows=rows, threads=2)
    return rows


def _worker(rank, world, port, rows, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from agi_lidar_slam_amd import shard
    sup = shard.super_sums(rows, rank, world)
    # a rank only touches its own shard of points
    b, e = shard.shard_range(rows.shape[0], rank, world)
    sup_local = shard.super_sums(np.where((np.arange(rows.shape[0]) >= b)[:, None]
                                          & (np.arange(rows.shape[0]) < e)[:, None], rows, 0.0),
                                 rank, world)
    assert np.array_equal(sup, sup_local)
    t = torch.from_numpy(sup.copy())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    if rank == 0:
        q.put(t.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_sums_bitwise_equal_single_rank(world):
    from agi_lidar_slam_amd import shard
    rows = _rows()
    ref = shard.super_sums(rows, 0, 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + world
    procs = [ctx.Process(target=_worker, args=(r, world, port, rows, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    np.testing.assert_array_equal(got, ref)
    a, b, m = shard.reduce_super(got)
    assert m == int(rows[:, 13].sum())


def test_shard_ranges_partition_the_scan():
    from agi_lidar_slam_amd import shard
    for n in [0, 1, 127, 128, 129, 1000, 100000, 100001]:
        for world in [1, 2, 4, 8]:
            spans = [shard.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
                assert e0 == b1 and b0 <= e0
