"""Point sharding and the fixed summation tree (mirror of csrc/slio_common.hpp).

The scan of n points is cut into C = ceil(n / 128) chunks; super-chunk s
(0..7) covers chunks [s*C//8, (s+1)*C//8); rank r of N (N | 8) owns
super-chunks [r*8/N, (r+1)*8/N).  Each rank writes its super-chunk sums and
zeros elsewhere, so a SUM all-reduce over ranks is an exact gather and the
final 8-term sum runs in the same order at every N: 1/2/4/8 GPUs give
bitwise-identical H^T H / H^T h.
"""
from __future__ import annotations

import numpy as np

CHUNK = 128
NSUPER = 8
NPROD = 91


def num_chunks(n: int) -> int:
    return (n + CHUNK - 1) // CHUNK


def super_lo(C: int, s: int) -> int:
    return (C * s) // NSUPER


def rank_chunks(n: int, rank: int, nranks: int) -> tuple[int, int]:
    if NSUPER % nranks:
        raise ValueError("nranks must divide 8")
    C = num_chunks(n)
    per = NSUPER // nranks
    return super_lo(C, rank * per), super_lo(C, (rank + 1) * per)


def shard_range(n: int, rank: int, nranks: int) -> tuple[int, int]:
    c0, c1 = rank_chunks(n, rank, nranks)
    return min(c0 * CHUNK, n), min(c1 * CHUNK, n)


def product_table() -> tuple[np.ndarray, np.ndarray]:
    pa, pb = [], []
    for i in range(12):
        for j in range(i, 12):
            pa.append(i)
            pb.append(j)
    for i in range(12):
        pa.append(i)
        pb.append(12)
    pa.append(13)
    pb.append(13)
    return np.array(pa), np.array(pb)


def super_sums(rows: np.ndarray, rank: int = 0, nranks: int = 1) -> np.ndarray:
    """Fixed-tree sums of per-point rows (n, 14) -> (8, 91); rows of
    super-chunks the rank does not own are zero (CPU model of the device
    reduction, used by the multi-rank tests)."""
    n = rows.shape[0]
    pa, pb = product_table()
    C = num_chunks(n)
    prod = rows[:, pa] * rows[:, pb]          # (n, 91)
    chunk = np.zeros((C, NPROD))
    for c in range(C):
        blk = prod[c * CHUNK:(c + 1) * CHUNK]
        acc = np.zeros(NPROD)
        for r in range(blk.shape[0]):         # fixed order within the chunk
            acc = acc + blk[r]
        chunk[c] = acc
    out = np.zeros((NSUPER, NPROD))
    per = NSUPER // nranks
    for s in range(rank * per, (rank + 1) * per):
        acc = np.zeros(NPROD)
        for c in range(super_lo(C, s), super_lo(C, s + 1)):
            acc = acc + chunk[c]
        out[s] = acc
    return out


def reduce_super(sup: np.ndarray) -> tuple[np.ndarray, np.ndarray, int]:
    tot = sup[0].copy()
    for s in range(1, NSUPER):
        tot = tot + sup[s]
    return tot[:78], tot[78:90], int(round(tot[90]))
