"""Node-shard geometry and the candidate exchange of the sharded engine.

The device path lives in ks_engine.cpp (ks_shard / ks_step): rank r scans its contiguous range
of 256-node blocks, merges it to an exact per-pod top-L list of packed keys, the lists are
all-gathered over RCCL, and a second merge gives the global top-L.  This module restates the
geometry (``part_blocks``, identical to ks_load_nodes) and the merge for the host side: the
bench uses it to describe a run and the CPU tests use it to check the exchange under gloo.
"""
from __future__ import annotations

import numpy as np

BLOCK_NODES = 256
TOP_L = 8


def engine_part_blocks(n_nodes: int, world: int, vshards: int = 1) -> np.ndarray:
    """The engine's own layout (include/ks_engine.h ks_shard_layout, used by ks_load_nodes)."""
    import ctypes as C
    from . import _lib
    out = np.zeros(world * vshards + 1, np.int32)
    rc = _lib.load().ks_shard_layout(n_nodes, world, vshards, out.ctypes.data_as(C.c_void_p))
    if rc != _lib.KS_OK:
        raise ValueError(f"ks_shard_layout({n_nodes}, {world}, {vshards}) = {rc}")
    return out.astype(np.int64)


def engine_merge(cand_all: np.ndarray) -> np.ndarray:
    """The engine's second merge on the host (ks_merge_candidates: the device merge's per-list
    step): cand_all[G][B][L] -> [B][L]."""
    import ctypes as C
    from . import _lib
    src = np.ascontiguousarray(cand_all, dtype=np.uint64)
    G, B, L = src.shape
    assert L == TOP_L
    out = np.zeros((B, L), np.uint64)
    rc = _lib.load().ks_merge_candidates(src.ctypes.data_as(C.c_void_p), G, B, out.ctypes.data_as(C.c_void_p))
    if rc != _lib.KS_OK:
        raise ValueError(f"ks_merge_candidates = {rc}")
    return out


def part_blocks(n_nodes: int, world: int, vshards: int = 1) -> np.ndarray:
    """Block boundaries of the world*vshards parts (ks_load_nodes: p * nblk / G)."""
    n_pad = max(64, (n_nodes + 63) // 64 * 64)
    nblk = (n_pad + BLOCK_NODES - 1) // BLOCK_NODES
    G = world * vshards
    return np.array([p * nblk // G for p in range(G + 1)], np.int64)


def rank_nodes(n_nodes: int, world: int, rank: int, vshards: int = 1) -> tuple[int, int]:
    """Node range [lo, hi) scanned by `rank`."""
    pb = part_blocks(n_nodes, world, vshards)
    lo = int(pb[rank * vshards]) * BLOCK_NODES
    hi = int(pb[(rank + 1) * vshards]) * BLOCK_NODES
    return min(lo, n_nodes), min(hi, n_nodes)


def packed_keys(total: np.ndarray, candidate: np.ndarray, node0: int = 0) -> np.ndarray:
    """(total + 1) << 32 | (0xFFFFFFFF - node); 0 for non-candidates (kubesim.go:208-222)."""
    node = np.arange(node0, node0 + len(total), dtype=np.uint64)
    k = ((total.astype(np.uint64) + np.uint64(1)) << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - node)
    return np.where(candidate, k, np.uint64(0))


def top_l(keys: np.ndarray, L: int = TOP_L) -> np.ndarray:
    """Sorted (descending) top-L of one pod's keys, zero-padded."""
    out = np.zeros(L, np.uint64)
    s = np.sort(keys[keys != 0])[::-1][:L]
    out[: len(s)] = s
    return out


def merge_lists(lists: np.ndarray, L: int = TOP_L) -> np.ndarray:
    """lists[G][B][L] -> [B][L]: the exact top-L of the union (the second merge)."""
    G, B, _ = lists.shape
    return np.stack([top_l(lists[:, b, :].reshape(-1), L) for b in range(B)])
