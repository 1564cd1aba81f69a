"""Build the in-tree native libraries.

``build()`` compiles ``agi_lidar_slam_amd/libslio.so`` (HIP kernels + C-ABI +
host IKF driver) for gfx950 with hipcc.  The library is built in-tree so it
travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

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
]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps += [os.path.join(ROOT, "include", h) for h in ("slio.h", "slio_frontend.h")]
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    cmd = [HIPCC, *FLAGS, "-I", os.path.join(ROOT, "include"), *srcs, "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
