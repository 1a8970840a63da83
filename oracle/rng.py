"""Counter-based dropout RNG, restated in numpy (TEST INFRASTRUCTURE ONLY).

The HIP kernels draw every dropout bit from ``pcv_hash3(seed, site, idx)``
(plaincv_amd/csrc/common.h).  This module reproduces the same 32-bit hash so
the oracle can apply bit-identical masks; the reference's threefry stream
(flax nn.Dropout / SelfAttention broadcast dropout) is not reproducible
without JAX, so only the *distribution* (Bernoulli(keep), inverted scaling
1/keep) is reference semantics — see SURVEY.md §7 hard part (vii).
"""
import numpy as np

_M32 = np.uint64(0xFFFFFFFF)


def hash3(seed: int, site: int, idx: np.ndarray) -> np.ndarray:
    """lowbias32 mix of (idx*G1 + site*G2 + seed*G3) mod 2^32, vectorised."""
    idx = np.asarray(idx, dtype=np.uint64) & _M32
    x = (idx * np.uint64(0x9E3779B1) + np.uint64((site * 0x85EBCA77) & 0xFFFFFFFF)
         + np.uint64((seed * 0xC2B2AE3D) & 0xFFFFFFFF)) & _M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & _M32
    x ^= x >> np.uint64(16)
    return x.astype(np.uint32)


def keep_threshold(rate: float) -> int:
    """Elements with hash >= threshold are kept (P(keep) = 1 - rate)."""
    t = int(rate * 4294967296.0)
    return min(max(t, 0), 0xFFFFFFFF)


def keep_mask(seed: int, site: int, shape, rate: float) -> np.ndarray:
    """Boolean keep mask for a row-major tensor of ``shape`` (flat index = idx)."""
    n = int(np.prod(shape))
    h = hash3(seed, site, np.arange(n, dtype=np.uint64))
    return (h >= np.uint32(keep_threshold(rate))).reshape(shape)
