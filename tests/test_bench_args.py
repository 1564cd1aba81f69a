"""bench.py's --gpus contract (CPU only: every case fails before anything
touches a GPU).  A run that cannot place one rank per GPU must exit non-zero
instead of printing a line measured on fewer GPUs than asked for."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    e.update(env)
    return subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=e, capture_output=True, text=True,
                          timeout=120)


def test_gpus_disagrees_with_world_size():
    r = _run(["--gpus", "2"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "disagrees with WORLD_SIZE=1" in r.stderr, r.stderr[-2000:]
    r = _run(["--gpus", "1"], WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "disagrees with WORLD_SIZE=4" in r.stderr, r.stderr[-2000:]


def test_gpus_more_than_visible():
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    r = _run(["--gpus", str(n)])
    assert r.returncode == 2 and f"needs {n} GPUs" in r.stderr, r.stderr[-2000:]
    # under torch.distributed.run: every local rank needs its own device (nccl)
    r = _run(["--gpus", str(n)], WORLD_SIZE=str(n), RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(n))
    assert r.returncode == 2 and f"need {n} GPUs" in r.stderr, r.stderr[-2000:]


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0"])
    assert r.returncode == 2 and "--gpus must be >= 1" in r.stderr, r.stderr[-2000:]
