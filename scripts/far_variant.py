"""Diagnostic: the inside-building far case (test_gpu_far) with a chosen
library build, one pass, timed, results checked vs the oracle.
usage: SLIO_LIB=path python scripts/far_variant.py [cell]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from agi_lidar_slam_amd import _lib as L, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

lib = L.load(os.environ.get("SLIO_LIB", L.LIB_PATH))
from test_gpu_parity import iterate, mk, results, state_of, upload_map, upload_scan  # noqa: E402
from test_gpu_far import far_count  # noqa: E402

cell = float(sys.argv[1]) if len(sys.argv) > 1 else 1.25
mp, fr = synth.make_problem(200000, 20000, pattern="avia", sensor="origin")
T = O.Tree(mp)
st = state_of(fr)
q = O.body_to_world(st, fr.body)
ridx, rsqd = T.knn(q, 5)
h = mk(L, cell=cell)
upload_map(L, h, mp)
upload_scan(L, h, fr.body)
print("lib", os.environ.get("SLIO_LIB"), "start", flush=True)
t0 = time.time()
iterate(L, h, st, True)
print("pass s", time.time() - t0, "far", far_count(L, h), flush=True)
idx, sqd, *_ = results(L, h, q.shape[0])
print("idx equal", np.array_equal(idx, ridx), "sqd equal", np.array_equal(sqd, rsqd), flush=True)
