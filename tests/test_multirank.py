"""World-size-2/4 gloo tests of the N>1 reduction path on CPU.

Each rank forms the super rows of its own super-chunks from the chunk
partials of its own chunks (tests/tree_model.py: the device's segment-row
tree, k_super_sums / fused_tail), zeros elsewhere; a SUM all-reduce must
reproduce the single-rank tree bit for bit, which is what makes 1/2/4/8-GPU
runs identical.  tests/test_gpu_parity.py::test_sharded_handles_bitwise_equal
pins the model to the device's own super rows."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import tree_model as TM  # noqa: E402


def _partials(n=5000, seed=1):
    from oracle import oracle as O
    from agi_lidar_slam_amd import synth
    mpts, fr = synth.make_problem(50000, n, seed=seed, pattern="avia")
    T = O.Tree(mpts)
    st = np.concatenate([fr.init_pos, fr.init_rot, [1, 0, 0, 0], synth.AVIA_T_LI, np.zeros(9),
                         [0, 0, -9.81]])
    ps = O.PassState(n)
    rows = np.zeros((n, 14))
    O.h_pass(T, st, fr.body, ps, True, rows=rows, threads=2)
    return TM.chunk_partials(rows)


def _worker(rank, world, port, part, q):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import tree_model as TM  # noqa: F811
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # a rank only reads its own chunks: the others are poisoned
    c0, c1 = TM.rank_chunks(part.shape[0] * TM.CHUNK, rank, world)
    mine = np.full_like(part, np.nan)
    mine[c0:c1] = part[c0:c1]
    sup = TM.super_rows(mine, rank, world)
    assert np.isfinite(sup).all()
    t = torch.from_numpy(sup.copy())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    if rank == 0:
        q.put(t.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_sums_bitwise_equal_single_rank(world):
    part = _partials()
    ref = TM.super_rows(part, 0, 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + world
    procs = [ctx.Process(target=_worker, args=(r, world, port, part, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    np.testing.assert_array_equal(got, ref)
    a, b, m = TM.reduce_super(got)
    assert m == int(round(part[:, 90].sum()))


def test_segment_rows_interleave_chunks():
    """Segment row g of super-chunk s takes chunks c0+g, c0+g+8, ... (not a
    contiguous run): with one-hot chunk partials each chunk lands in exactly
    the segment the device sums it in."""
    C = 100
    part = np.zeros((C, TM.NPROD))
    part[np.arange(C), np.arange(C) % TM.NPROD] = np.arange(1, C + 1)
    for s in range(TM.NSUPER):
        seg = TM.segment_rows(part, s)
        c0, c1 = TM.super_lo(C, s), TM.super_lo(C, s + 1)
        for c in range(c0, c1):
            assert seg[(c - c0) % TM.NSEG, c % TM.NPROD] == c + 1


def test_shard_ranges_partition_the_scan():
    for n in [0, 1, 127, 128, 129, 1000, 100000, 100001]:
        for world in [1, 2, 4, 8]:
            spans = [TM.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
                assert e0 == b1 and b0 <= e0
