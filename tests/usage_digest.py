"""Test helper: the per-tick usage digest of include/ks_engine.h (ks_usage_digest) recomputed
from full [T][n][3] usage matrices (the oracle's), with the node weight written out here
independently of the engine (ks_node_mix)."""
import numpy as np

M64 = (1 << 64) - 1


def node_mix(node: int) -> int:
    z = ((node + 1) * 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def digest_from_matrices(u):
    """u: [T][n][3] int64 usage per tick -> [T][6] uint64 digest."""
    T, n, _ = u.shape
    w = np.array([node_mix(i) for i in range(n)], dtype=np.uint64)
    out = np.zeros((T, 6), np.uint64)
    uu = u.astype(np.uint64)
    with np.errstate(over="ignore"):
        out[:, 0:3] = uu.sum(axis=1, dtype=np.uint64)
        out[:, 3:6] = (uu * w[None, :, None]).sum(axis=1, dtype=np.uint64)
    return out
