"""CPU checks of the device evaluator's integer math (ks_device.h compiled for the host).

* narrow (32-bit, float-estimate + exact correction) LeastRequested / BalancedAllocation floors
  against exact integer arithmetic;
* narrow total == wide total wherever the narrow evaluator is selected (capacities < 2^29);
* the resolver's float prune bound never undercuts the exact total (prune_tmax >= total) and is
  tight (equal to it but for values within the float slack of an integer).

The device build replaces the host's exact reciprocal by v_rcp (~1 ulp); the margins cover
both, and the GPU parity suites check the device build end to end.
"""
import ctypes as C
import math
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "eval_host.cpp")
DEV_H = os.path.join(HERE, "..", "kubernetes-simulator_amd", "csrc", "ks_device.h")
LIB = os.path.join(HERE, "native", "libks_hosteval.so")


class Cfg(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("nwb", C.c_int32), ("filter_feeds", C.c_int32),
                ("filters", C.c_uint32), ("has_scorers", C.c_int32), ("w_lr", C.c_int32),
                ("w_ba", C.c_int32), ("const_total", C.c_int32), ("tick_seconds", C.c_int32),
                ("pad_", C.c_int32)]


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(SRC), os.path.getmtime(DEV_H)):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", LIB, SRC],
                       check=True)
    L = C.CDLL(LIB)
    p = lambda: C.c_void_p
    L.ks_host_lr_n_batch.argtypes = [C.c_int64] + [p()] * 3
    L.ks_host_ba_n_batch.argtypes = [C.c_int64] + [p()] * 5
    L.ks_host_ba_batch.argtypes = [C.c_int64] + [p()] * 5
    L.ks_host_prune_batch.argtypes = [C.POINTER(Cfg), C.c_int64] + [p()] * 7
    return L


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _lr_exact(A, u):
    A = A.astype(np.int64); u = u.astype(np.int64)
    out = np.zeros(len(A), np.int64)
    ok = (A > 0) & (u <= A)
    out[ok] = ((A[ok] - u[ok]) * 10) // A[ok]
    return out


def _ba_exact(Ac, Am, uc, um):
    Ac = [int(x) for x in Ac]; Am = [int(x) for x in Am]; uc = [int(x) for x in uc]; um = [int(x) for x in um]
    out = []
    for a, b, x, y in zip(Ac, Am, uc, um):
        if a <= 0 or b <= 0 or x >= a or y >= b:
            out.append(0)
            continue
        D = a * b
        X = abs(x * b - y * a)
        out.append((10 * (D - X)) // D)
    return np.array(out, np.int64)


def _narrow_cases(rng, n):
    A = rng.integers(1, 1 << 29, n).astype(np.int32)
    # bias towards the floor boundaries: u = A - k*A/10 +- small
    k = rng.integers(0, 11, n)
    jitter = rng.integers(-3, 4, n)
    u = np.clip(A.astype(np.int64) - (k * A.astype(np.int64)) // 10 + jitter, 0, (1 << 30)).astype(np.int32)
    rnd = rng.random(n) < 0.3
    u[rnd] = rng.integers(0, 1 << 29, rnd.sum()).astype(np.int32)
    return A, u


def test_lr_narrow_exact(lib):
    rng = np.random.default_rng(11)
    A, u = _narrow_cases(rng, 200_000)
    out = np.zeros(len(A), np.int32)
    lib.ks_host_lr_n_batch(len(A), _p(A), _p(u), _p(out))
    np.testing.assert_array_equal(out, _lr_exact(A, u))


def test_ba_narrow_exact(lib):
    rng = np.random.default_rng(12)
    n = 60_000
    Ac, uc = _narrow_cases(rng, n)
    Am, um = _narrow_cases(rng, n)
    # balanced cases: um/Am close to uc/Ac (X small, BA near 10)
    bal = rng.random(n) < 0.3
    um[bal] = np.clip((uc[bal].astype(np.int64) * Am[bal]) // Ac[bal] + rng.integers(-2, 3, bal.sum()),
                      0, (1 << 30)).astype(np.int32)
    out = np.zeros(n, np.int32)
    lib.ks_host_ba_n_batch(n, _p(Ac), _p(Am), _p(uc), _p(um), _p(out))
    np.testing.assert_array_equal(out, _ba_exact(Ac, Am, uc, um))


def test_ba_wide_exact(lib):
    rng = np.random.default_rng(13)
    n = 40_000
    Ac = rng.integers(1, 1 << 58, n, dtype=np.int64)
    Am = rng.integers(1, 1 << 58, n, dtype=np.int64)
    uc = (Ac * rng.random(n)).astype(np.int64)
    um = (Am * rng.random(n)).astype(np.int64)
    out = np.zeros(n, np.int32)
    lib.ks_host_ba_batch(n, _p(Ac), _p(Am), _p(uc), _p(um), _p(out))
    np.testing.assert_array_equal(out, _ba_exact(Ac, Am, uc, um))


def _nodes(rng, n, cap_bits):
    alloc = np.zeros((n, 4), np.int64)
    for k in range(3):
        alloc[:, k] = rng.integers(0, 1 << cap_bits, n)
    alloc[rng.random(n) < 0.05, 0] = -1
    alloc[rng.random(n) < 0.05, 1] = -1
    alloc[rng.random(n) < 0.05, 1] = 0
    alloc[:, 3] = 110
    run = np.zeros((n, 3), np.int64)
    for k in range(3):
        frac = rng.random(n) ** 0.5
        run[:, k] = np.maximum(alloc[:, k], 0) * frac
    req = np.zeros((n, 3), np.int64)
    for k in range(3):
        req[:, k] = (np.maximum(alloc[:, k], 1) * rng.random(n) ** 3 * 0.5).astype(np.int64)
    req[rng.random(n) < 0.1, 0] = 0
    return alloc, run, req


@pytest.mark.parametrize("feeds,const,w_lr,w_ba", [(1, 0, 1, 1), (0, 0, 1, 1), (1, 5, 2, 0), (0, 3, 0, 3),
                                                   (1, 0, 7, 13), (0, 1000, 50, 50)])
@pytest.mark.parametrize("cap_bits", [20, 28])
def test_prune_bound_sound(lib, feeds, const, w_lr, w_ba, cap_bits):
    rng = np.random.default_rng(cap_bits * 1000 + w_lr * 10 + w_ba + const)
    n = 50_000
    alloc, run, req = _nodes(rng, n, cap_bits)
    c = Cfg(n_nodes=n, nwb=0, filter_feeds=feeds, filters=1 if feeds else 0, has_scorers=1, w_lr=w_lr,
            w_ba=w_ba, const_total=const, tick_seconds=1)
    t1 = np.zeros(n, np.uint32); t1n = np.zeros(n, np.uint32); tm = np.zeros(n, np.uint32)
    t1t = np.zeros(n, np.uint32)
    lib.ks_host_prune_batch(C.byref(c), n, _p(alloc), _p(run), _p(req), _p(t1), _p(t1n), _p(tm), _p(t1t))
    np.testing.assert_array_equal(t1n, t1)  # narrow == wide below 2^29
    live = t1 > 0
    assert live.sum() > n // 3
    total = t1[live].astype(np.int64) - 1
    assert (total <= tm[live].astype(np.int64)).all(), "prune bound below the exact total"
    # and the bound is useful: mostly within a couple of points of the exact total
    assert np.mean(tm[live].astype(np.int64) - total) < 0.2 * (w_lr + w_ba) + 0.5


@pytest.mark.parametrize("feeds,const,w_lr,w_ba", [(1, 0, 1, 1), (0, 0, 1, 1), (1, 5, 2, 0), (0, 3, 0, 3)])
@pytest.mark.parametrize("cap_bits", [6, 11, 13])
def test_tiny_eval_exact(lib, feeds, const, w_lr, w_ba, cap_bits):
    """eval_total1_tiny == the wide evaluator while capacities and Ac*Am stay below 2^26,
    including C3-like small-denominator states (exact integer LR / BA values)."""
    rng = np.random.default_rng(1000 + cap_bits * 7 + w_lr * 3 + w_ba + const + feeds)
    n = 80_000
    alloc, run, req = _nodes(rng, n, cap_bits)
    # C3-like: multiples of small units, requests up to the capacity and beyond (clamp path)
    run[:, :2] = (run[:, :2] // 8) * 8
    req[rng.random(n) < 0.05, 0] = 1 << 40
    req[rng.random(n) < 0.05, 1] = (1 << 27) + 5
    assert (np.maximum(alloc[:, 0], 0) * np.maximum(alloc[:, 1], 0) < (1 << 26)).all()
    c = Cfg(n_nodes=n, nwb=0, filter_feeds=feeds, filters=1 if feeds else 0, has_scorers=1, w_lr=w_lr,
            w_ba=w_ba, const_total=const, tick_seconds=1)
    t1 = np.zeros(n, np.uint32); t1n = np.zeros(n, np.uint32); tm = np.zeros(n, np.uint32)
    t1t = np.zeros(n, np.uint32)
    lib.ks_host_prune_batch(C.byref(c), n, _p(alloc), _p(run), _p(req), _p(t1), _p(t1n), _p(tm), _p(t1t))
    np.testing.assert_array_equal(t1t, t1)


@pytest.mark.parametrize("feeds,filters,const,w_lr,w_ba", [(1, 7, 0, 1, 1), (0, 0, 0, 1, 1), (1, 1, 5, 2, 0),
                                                           (0, 0, 3, 0, 3), (1, 7, 0, 7, 13),
                                                           (1, 3, 1000, (1 << 24) - 1, 50)])
@pytest.mark.parametrize("cap_bits", [4, 11, 12])
def test_micro_eval_exact(lib, feeds, filters, const, w_lr, w_ba, cap_bits):
    """eval_total1_micro == the wide evaluator on the micro domain (capacities < 2^16, Ac*Am < 2^24,
    weights < 2^24): fit boundaries (free amount 0 / -1), absent (-1) and zero capacities, absent
    request keys, clamped requests, the pods capacity and the taint / selector masks."""
    rng = np.random.default_rng(5000 + cap_bits * 11 + w_lr % 97 * 3 + w_ba + const + filters)
    n = 100_000
    alloc, run3, req = _nodes(rng, n, cap_bits)
    alloc[:, 3] = rng.integers(0, 4, n)
    run = np.zeros((n, 4), np.int64)
    run[:, :3] = run3
    run[:, 3] = rng.integers(0, 4, n)
    # exact-fit and one-over boundaries, C3-like unit multiples, clamp path
    for k in range(3):
        cap = np.maximum(alloc[:, k], 0)
        edge = rng.random(n) < 0.15
        req[edge, k] = np.maximum(cap[edge] - run[edge, k] + rng.integers(-1, 2, edge.sum()), 0)
    req[rng.random(n) < 0.03, 0] = 1 << 40
    req[rng.random(n) < 0.03, 1] = (1 << 17) + 5
    req[rng.random(n) < 0.03, 2] = (1 << 17) - 1
    assert (np.maximum(alloc[:, 0], 0) * np.maximum(alloc[:, 1], 0) < (1 << 24)).all()
    keymask = rng.integers(0, 8, n).astype(np.uint32)
    masks = np.zeros((n, 4), np.uint64)
    bits = lambda p: np.where(rng.random(n) < p, np.uint64(1) << rng.integers(0, 64, n).astype(np.uint64), np.uint64(0))
    masks[:, 0] = bits(0.3) | bits(0.2)  # node taints
    masks[:, 1] = bits(0.5) | bits(0.5)  # node labels
    masks[:, 2] = masks[:, 0] | bits(0.3)  # tolerations: usually all
    masks[rng.random(n) < 0.2, 2] = 0
    masks[:, 3] = np.where(rng.random(n) < 0.5, masks[:, 1] & bits(1.0), bits(0.2))  # selectors
    c = Cfg(n_nodes=n, nwb=0, filter_feeds=feeds, filters=filters, has_scorers=1, w_lr=w_lr,
            w_ba=w_ba, const_total=const, tick_seconds=1)
    t1 = np.zeros(n, np.uint32); t1m = np.zeros(n, np.uint32)
    lib.ks_host_micro_batch.argtypes = [C.POINTER(Cfg), C.c_int64] + [C.c_void_p] * 7
    lib.ks_host_micro_batch(C.byref(c), n, _p(alloc), _p(run), _p(req), _p(keymask), _p(masks), _p(t1), _p(t1m))
    assert (t1 > 0).sum() > n // 10
    np.testing.assert_array_equal(t1m, t1)
    # the scan's form (per-pod ScanRec: clamped / fit-biased requests, complemented tolerations)
    t1s = np.zeros(n, np.uint32)
    lib.ks_host_scan_micro_batch.argtypes = [C.POINTER(Cfg), C.c_int64] + [C.c_void_p] * 6
    lib.ks_host_scan_micro_batch(C.byref(c), n, _p(alloc), _p(run), _p(req), _p(keymask), _p(masks), _p(t1s))
    np.testing.assert_array_equal(t1s, t1)
    c.has_scorers = 0  # no scorer: no candidate
    lib.ks_host_scan_micro_batch(C.byref(c), n, _p(alloc), _p(run), _p(req), _p(keymask), _p(masks), _p(t1s))
    assert (t1s == 0).all()
