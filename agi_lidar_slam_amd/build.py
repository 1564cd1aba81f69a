"""Build the in-tree native libraries.

``build()`` compiles ``agi_lidar_slam_amd/libslio.so`` (HIP kernels + C-ABI +
host IKF driver) for gfx950 with hipcc.  The library is built in-tree so it
travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libslio.so")

SOURCES = ["slio_device.hip", "slio_ikf.cpp", "slio_imu.cpp", "slio_s2m.cpp", "slio_lio.hip"]
HEADERS = ["slio_common.hpp", "slio_plane.hpp", "slio_so3.hpp"]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    # exact IEEE evaluation order: parity with the CPU oracle is bitwise
    "-ffp-contract=off",
    "-fno-fast-math",
    "-Wall",
    # the in-library all-reduce of the multi-GPU path (RCCL over xGMI)
    "-L/opt/rocm/lib",
    "-lrccl",
    "-Wl,-rpath,/opt/rocm/lib",
]


def _deps() -> list[str]:
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return deps + [os.path.join(ROOT, "include", h) for h in ("slio.h", "slio_frontend.h")]


def source_hash() -> str:
    """16 hex digits of a SHA-256 over the library's sources and headers; the
    library reports the digest it was compiled with (slio_build_id)."""
    h = hashlib.sha256()
    for d in _deps():
        if os.path.exists(d):
            h.update(os.path.basename(d).encode())
            h.update(open(d, "rb").read())
    return h.hexdigest()[:16]


def _stale() -> bool:
    """The library is stale unless it carries the digest of the current
    sources (slio_build_id's string is embedded in the binary); file times
    are not trusted, as a copy or checkout changes them."""
    if not os.path.exists(LIB):
        return True
    with open(LIB, "rb") as f:
        return source_hash().encode() not in f.read()


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every source to an object in parallel (the two HIP files take
    most of the time), then link the shared library."""
    if not force and not _stale():
        return LIB
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    tag = source_hash()
    compile_flags = [f for f in FLAGS if f != "-shared" and not f.startswith(("-L", "-l", "-Wl"))]
    objs, procs = [], []
    for src in srcs:
        obj = os.path.join(PKG, "_obj", os.path.basename(src) + ".o")
        os.makedirs(os.path.dirname(obj), exist_ok=True)
        cmd = [HIPCC, *compile_flags, f'-DSLIO_SOURCE_HASH="{tag}"', "-I", os.path.join(ROOT, "include"),
               "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    failed = [cmd for p, cmd in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    link = [HIPCC, *FLAGS, *objs, "-o", LIB + ".tmp"]
    subprocess.run(link, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
