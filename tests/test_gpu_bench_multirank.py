"""bench.py's multi-rank path (C4: scan points sharded over ranks, one
all-reduce of the 8 x 91 super-chunk sums per IKF iteration through the
library's reduce hook) run end to end with torch.distributed: 2 ranks on the
box's one GPU over gloo (RCCL refuses two ranks on one device; the hook, the
shared stream and the device-resident update are the same).  The sharded run
must end with the single-rank x and P bit for bit (result_digest: SHA-256 of
the last update's x and P) and select the same effective points."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--map-points", "200000", "--scan-points", "20000", "--steps", "5", "--warmup", "2",
         "--no-cpu-baseline"]


def _run(cmd):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_two_ranks_gloo_matches_single():
    one = _run([sys.executable, "bench.py", *SMALL])
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", "29541", "bench.py", "--gpus", "2",
                "--dist-backend", "gloo", *SMALL])
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["value"] > 0
    assert two["config"]["effective_points"] == one["config"]["effective_points"]
    assert two["result_digest"] == one["result_digest"]


def test_bench_gpus_spawns_its_ranks():
    """A plain `bench.py --gpus 2` (no torch.distributed.run around it) starts
    its two ranks itself, one process each, before touching a GPU: the same
    line as the driver's torchrun launch (gloo here: the box has one GPU)."""
    one = _run([sys.executable, "bench.py", *SMALL])
    two = _run([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", *SMALL])
    assert two["n_gpus"] == 2 and two["value"] > 0
    assert two["result_digest"] == one["result_digest"]


def test_bench_reference_flow_line():
    """--mode reference --iters 3 (the drop-in's control flow, mapping_avia.launch:11):
    a bench line whose passes include reuse passes, with a roofline."""
    ref = _run([sys.executable, "bench.py", *SMALL, "--mode", "reference", "--iters", "3"])
    cfg = ref["config"]
    assert cfg["control_flow"] == "reference" and cfg["maximum_iter"] == 3
    assert 1 <= cfg["searches_per_step"] <= cfg["iterations_per_step"] <= 4
    assert ref["value"] > 0 and ref["roofline"]["achieved"] > 0
