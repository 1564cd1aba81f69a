"""Test model of the device's point sharding and fixed summation tree
(csrc/slio_common.hpp rank_chunks / super_lo; slio_device.hip k_super_sums
and fused_tail).  Test infrastructure only: the product never imports it.

The scan of n points is cut into C = ceil(n / 128) chunks, each summed by one
workgroup into a 91-double chunk partial (its rounding is the matrix cores',
so the model starts from the chunk partials).  Super-chunk s (0..7) covers
chunks [s*C//8, (s+1)*C//8); segment row g of super-chunk s sums its chunks
c0+g, c0+g+8, ... in that order; super row s is segment rows 0..7 of s in
order; the pass total is super rows 0..7 in order.  Rank r of N (N | 8) owns
super-chunks [r*8/N, (r+1)*8/N) and writes zeros for the others, so a SUM
all-reduce over ranks is an exact gather: 1/2/4/8 ranks give bitwise-
identical H^T H / H^T h.
"""
from __future__ import annotations

import numpy as np

CHUNK = 128
NSUPER = 8
NSEG = 8          # segment rows per super-chunk
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


def chunk_partials(rows: np.ndarray) -> np.ndarray:
    """Per-chunk products of per-point rows (n, 14) -> (C, 91), rows summed in
    order (a stand-in for the device's matrix-core chunk sums)."""
    n = rows.shape[0]
    pa, pb = product_table()
    prod = rows[:, pa] * rows[:, pb]
    C = num_chunks(n)
    out = np.zeros((C, NPROD))
    for c in range(C):
        acc = np.zeros(NPROD)
        for r in prod[c * CHUNK:(c + 1) * CHUNK]:
            acc = acc + r
        out[c] = acc
    return out


def segment_rows(part: np.ndarray, s: int) -> np.ndarray:
    """The 8 segment rows of super-chunk s: row g sums chunks c0+g, c0+g+8, ...
    in order (k_super_sums / fused_tail)."""
    C = part.shape[0]
    c0, c1 = super_lo(C, s), super_lo(C, s + 1)
    seg = np.zeros((NSEG, NPROD))
    for g in range(NSEG):
        acc = np.zeros(NPROD)
        for c in range(c0 + g, c1, NSEG):
            acc = acc + part[c]
        seg[g] = acc
    return seg


def super_rows(part: np.ndarray, rank: int = 0, nranks: int = 1) -> np.ndarray:
    """The (8, 91) super rows a rank writes from the chunk partials of its own
    chunks (zeros for super-chunks it does not own)."""
    out = np.zeros((NSUPER, NPROD))
    per = NSUPER // nranks
    for s in range(rank * per, (rank + 1) * per):
        seg = segment_rows(part, s)
        acc = seg[0].copy()
        for g in range(1, NSEG):
            acc = acc + seg[g]
        out[s] = acc
    return out


def reduce_super(sup: np.ndarray) -> tuple[np.ndarray, np.ndarray, int]:
    tot = sup[0].copy()
    for s in range(1, NSUPER):
        tot = tot + sup[s]
    return tot[:78], tot[78:90], int(round(tot[90]))
