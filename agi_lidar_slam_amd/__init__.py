"""MI355X-native IKF scan-matching core for S-FAST_LIO laserMapping.

The device path lives in ``libslio.so`` (HIP kernels + C-ABI, include/slio.h);
``esekf`` mirrors the reference's ``esekfom::esekf`` interface on top of it.
"""
__all__ = ["build", "synth"]
