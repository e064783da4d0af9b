"""ctypes wrapper for the C oracle (oracle/libks_oracle.so).  TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libks_oracle.so")


def build(force=False):
    src = os.path.join(HERE, "ks_oracle.c")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-C", HERE, "-s"])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        p = C.c_void_p
        L.ko_create.restype = p
        L.ko_create.argtypes = [p, C.c_int64, p, p, p, p, p, p]
        L.ko_destroy.argtypes = [p]
        L.ko_submit.argtypes = [p, C.c_int64] + [p] * 13
        L.ko_step.argtypes = [p, C.c_int64, p, p, p, p, C.c_int64, p]
        L.ko_usage.argtypes = [p, p]
        L.ko_eval.argtypes = [p, C.c_int64, p, p]
        L.ko_set_threads.argtypes = [p, C.c_int]
        L.ko_tick.restype = C.c_int64
        L.ko_tick.argtypes = [p]
        L.ko_last_error.restype = C.c_char_p
        L.ko_last_error.argtypes = [p]
        _lib = L
    return _lib


class KoConfig(C.Structure):
    _fields_ = [("tick_seconds", C.c_int32), ("filter_mode", C.c_int32), ("filters", C.c_uint32),
                ("n_scorers", C.c_int32), ("scorer_kind", C.c_int32 * 8),
                ("scorer_weight", C.c_int32 * 8), ("scorer_value", C.c_int32 * 8)]


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class COracle:
    """CPU restatement of KubeSim (kubesim/kubesim.go) driven tick by tick."""

    def __init__(self, trace, *, filter_mode=0, filters=0, scorers=((0, 1, 1),)):
        cfg = KoConfig()
        cfg.tick_seconds = trace["tick_seconds"]
        cfg.filter_mode = filter_mode
        cfg.filters = filters
        cfg.n_scorers = len(scorers)
        for i, (k, w, v) in enumerate(scorers):
            cfg.scorer_kind[i], cfg.scorer_weight[i], cfg.scorer_value[i] = k, w, v
        nd = trace["nodes"]
        self.n = nd["n"]
        self._keep = [_c(nd["alloc"], np.int64), _c(nd["alloc_has"], np.uint8),
                      _c(nd["taint_off"], np.int32), _c(nd["taint"], np.int32),
                      _c(nd["label_off"], np.int32), _c(nd["label"], np.int32)]
        self.h = lib().ko_create(C.byref(cfg), self.n, *[_ptr(a) for a in self._keep])
        if not self.h:
            raise ValueError("ko_create refused the configuration (tick_seconds must be >= 1)")
        self.m = 0

    def set_threads(self, n: int):
        """Run the per-node loops on n OpenMP threads (identical results)."""
        lib().ko_set_threads(self.h, int(n))

    def close(self):
        if getattr(self, "h", None):
            lib().ko_destroy(self.h)
            self.h = None

    __del__ = close

    def submit(self, trace):
        p = trace["pods"]
        arrs = [_c(p["arrival"], np.int64), _c(p["req"], np.int64), _c(p["req_has"], np.uint8),
                _c(p["tol_off"], np.int32), _c(p["tol"], np.int32), _c(p["sel_off"], np.int32),
                _c(p["sel"], np.int32), _c(p["phase_off"], np.int32), _c(p["phase_sec"], np.int32),
                _c(p["phase_use"], np.int64), _c(p["phase_has"], np.uint8), _c(p["key_id"], np.int64),
                _c(p["flags"], np.uint8)]
        rc = lib().ko_submit(self.h, p["m"], *[_ptr(a) for a in arrs])
        if rc:
            raise ValueError(lib().ko_last_error(self.h).decode())
        self.m += p["m"]

    def step(self, ticks, cap=None):
        cap = ticks if cap is None else cap
        pod = np.zeros(cap, np.int64)
        node = np.zeros(cap, np.int32)
        tick = np.zeros(cap, np.int64)
        st = np.zeros(cap, np.int32)
        n = C.c_int64(0)
        rc = lib().ko_step(self.h, ticks, _ptr(pod), _ptr(node), _ptr(tick), _ptr(st), cap, C.byref(n))
        k = min(n.value, cap)
        return dict(pod=pod[:k], node=node[:k], tick=tick[:k], status=st[:k]), rc

    def usage(self):
        out = np.zeros((self.n, 3), np.int64)
        lib().ko_usage(self.h, _ptr(out))
        return out

    def eval(self, pod):
        feas = np.zeros(self.n, np.uint8)
        score = np.zeros(self.n, np.int64)
        rc = lib().ko_eval(self.h, pod, _ptr(feas), _ptr(score))
        assert rc == 0
        return feas, score

    @property
    def tick(self):
        return lib().ko_tick(self.h)

    def last_error(self):
        return lib().ko_last_error(self.h).decode()
