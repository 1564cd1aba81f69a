"""Diagnostic / A-B builds of libslio for scripts -- not product code.

The product loader (``agi_lidar_slam_amd._lib.load``) binds only
``agi_lidar_slam_amd/libslio.so`` and refuses one whose build id is not the
digest of the current sources.  A script that wants another build (a stamp
build from ``scripts/build_variant.sh``, or an earlier tree for a same-box A/B)
binds it here first; entry points an older build predates stay unbound.

  python scripts/variant.py LIB.so SCRIPT.py [ARGS...]   # run SCRIPT against LIB
  from variant import use; lib = use(path)               # inside a script
"""
from __future__ import annotations

import ctypes as C
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def use(path: str) -> C.CDLL:
    # torch first, as in the product scripts: its HIP runtime must be the one
    # loaded when the library's dependency resolves (the other order leaves
    # torch with "No HIP GPUs are available")
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    from agi_lidar_slam_amd import _lib as L
    if L._lib is not None:
        raise RuntimeError("a library is already bound in this process")
    lib = C.CDLL(os.path.abspath(path))
    for name, (res, args) in L.SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
    L._lib = lib
    print(f"[variant] {path} (build {lib.slio_build_id().decode()})", file=sys.stderr)
    return lib


if __name__ == "__main__":
    if len(sys.argv) < 3:
        sys.exit(__doc__)
    use(sys.argv[1])
    script = sys.argv[2]
    sys.argv = sys.argv[2:]
    sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
    runpy.run_path(script, run_name="__main__")
