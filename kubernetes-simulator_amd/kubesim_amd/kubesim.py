"""KubeSim's Run loop over the device engine — the Python twin of the Go drop-in
(go/kubesim/engine/kubesim.go), so the drop-in's call sequence can be run and timed where no Go
toolchain exists.

Reference: ``KubeSim.Run`` (kubesim/kubesim.go:90-123) calls every registered submitter in
order at each tick (``submit``, kubesim.go:126-139; ``api.Submitter``, api/submitter.go:10-16),
appends their pods FIFO and schedules one queued pod (``scheduleOne``, kubesim.go:143-166).

* :meth:`KubeSim.run` is that loop literally, as the Go shim's ``Run`` issues it: per tick the
  submitters' pods go to ``ks_submit_pods`` with arrival = the tick, then ``ks_step(1)``.  An
  optional ``probe`` runs the ``api.Filter`` / ``api.Scorer`` adapters (``ks_filter`` /
  ``ks_score``) on the queue's head pod each tick, as a plugin host would.
* :meth:`KubeSim.run_windowed` is the Go shim's ``RunWindowed``: for submitters that declare
  ``placement_blind = True`` (their output never depends on placements, like the reference
  example's, examples/main.go:96-128) the submitters are called for the next ``window`` ticks
  first, then one ``ks_step(window)``.  Binds, ticks and errors are identical to :meth:`run` —
  a pod's placement depends only on pods submitted before it, and each submit precedes the step
  that binds it (tests/test_dropin_gpu.py checks both against the oracle).

A submitter is a callable ``submit(tick, clock_seconds) -> encoded pods | None`` (the
``kubesim_amd.encode.encode_pods`` form; its ``arrival`` is overwritten with the tick).
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import _lib
from .engine import Engine, KsError, _c, _p


def slice_encoded(pods: dict, lo: int, hi: int) -> dict:
    """Encoded pods ``[lo, hi)`` (the phase CSR re-based)."""
    a, b = int(pods["phase_off"][lo]), int(pods["phase_off"][hi])
    out = dict(m=hi - lo, phase_off=(pods["phase_off"][lo:hi + 1] - a).astype(np.int32),
               phase_sec=pods["phase_sec"][a:b], phase_use=np.asarray(pods["phase_use"]).reshape(-1, 3)[a:b])
    for k in ("arrival", "req", "keymask", "tol", "sel", "flags"):
        out[k] = pods[k][lo:hi]
    out["key_id"] = pods["key_id"][lo:hi] if pods.get("key_id") is not None else None
    return out


class TraceSubmitter:
    """A submitter replaying a trace: at tick t it returns the pods whose arrival tick is t
    (their arrival is where the trace's own submitter would have returned them)."""

    placement_blind = True

    def __init__(self, enc_pods: dict):
        self.p = enc_pods
        self.arr = np.asarray(enc_pods["arrival"], np.int64)
        self.next = 0

    def __call__(self, tick: int, clock_seconds: int):
        lo = self.next
        hi = int(np.searchsorted(self.arr, tick, side="right"))
        if hi <= lo:
            return None
        self.next = hi
        return slice_encoded(self.p, lo, hi)


class KubeSim:
    """``kubesim.KubeSim`` with the scheduling loop on the device (one engine, one cluster)."""

    def __init__(self, engine: Engine, tick_seconds: int):
        self.eng = engine
        self.tick_seconds = tick_seconds
        self.submitters = []
        self.tick = engine.tick
        self.binds = []
        self.calls = {"submit": 0, "step": 0, "probe": 0}

    def register_submitter(self, s):
        """RegisterSubmitter (kubesim/kubesim.go:73-76)."""
        self.submitters.append(s)

    def _submit(self, t: int):
        for s in self.submitters:
            pods = s(t, t * self.tick_seconds)
            if pods is None or int(pods["m"]) == 0:
                continue
            pods = dict(pods)
            pods["arrival"] = np.full(int(pods["m"]), t, np.int64)
            self.eng.submit(pods)
            self.calls["submit"] += 1

    def _step(self, ticks: int):
        if ticks <= 0:
            return
        try:
            b = self.eng.step(ticks)
        except KsError as ex:
            if ex.binds is not None and len(ex.binds):
                self.binds.append(ex.binds)
            raise
        finally:
            self.calls["step"] += 1
        if len(b):
            self.binds.append(b)

    def run(self, ticks: int, probe=None):
        """``Run`` for ``ticks`` ticks: per tick submit (arrival = tick), then ``ks_step(1)``.
        ``probe(engine, tick)`` (optional) runs after the submit, before the step — the place an
        ``api.Filter`` / ``api.Scorer`` host would evaluate the queue's head pod."""
        for _ in range(ticks):
            self.tick += 1
            self._submit(self.tick)
            if probe is not None:
                probe(self.eng, self.tick)
                self.calls["probe"] += 1
            self._step(1)

    def run_windowed(self, ticks: int, window: int):
        """``RunWindowed``: submitters for the next ``window`` ticks, then one ``ks_step``."""
        if any(not getattr(s, "placement_blind", False) for s in self.submitters):
            raise ValueError("run_windowed: every submitter must be placement_blind")
        end = self.tick + ticks
        while self.tick < end:
            k = min(window, end - self.tick)
            for _ in range(k):
                self.tick += 1
                try:
                    self._submit(self.tick)
                except Exception:
                    # Run would have scheduled ticks < t before calling the submitters at t (the
                    # Go shim's RunWindowed does the same)
                    self._step(self.tick - 1 - self.eng.tick)
                    raise
            self._step(self.tick - self.eng.tick)

    def all_binds(self):
        if not self.binds:
            return np.zeros(0, dtype=[("pod", "<i8"), ("node", "<i4"), ("status", "<i4"), ("tick", "<i8")])
        return np.concatenate(self.binds)


class NativeRun:
    """``KubeSim.Run`` as the C++ host runs it (include/ks_kubesim.h, libks_kubesim.so): a trace
    submitter replayed natively, per tick ``ks_submit_pods`` + ``ks_step(1)`` (``window`` = 1) or
    ``RunWindowed`` (one ``ks_step(window)`` after ``window`` ticks of submits) — the call sequence
    of the cgo shim without any Python between the calls."""

    def __init__(self, engine: Engine, enc_pods: dict, tick_seconds: int):
        self.eng = engine
        self.L = _lib.load_run()
        self._keep = [_c(enc_pods["arrival"], np.int64), _c(enc_pods["req"], np.int64).reshape(-1, 3),
                      _c(enc_pods["keymask"], np.uint8), _c(enc_pods["tol"], np.uint64),
                      _c(enc_pods["sel"], np.uint64), _c(enc_pods["phase_off"], np.int32),
                      _c(enc_pods["phase_sec"], np.int32), _c(enc_pods["phase_use"], np.int64).reshape(-1, 3),
                      _c(enc_pods["flags"], np.uint8)]
        keys = enc_pods.get("key_id")
        self._keys = _c(keys, np.int64) if keys is not None else None
        t = _lib.KsPods(int(enc_pods["m"]), *[_p(a) for a in self._keep],
                        _p(self._keys) if self._keys is not None else None)
        self.sub = _lib.KsTraceSubmitter(t, 0, tick_seconds)
        self._fn = (C.c_void_p * 1)(C.cast(self.L.ks_trace_submit, C.c_void_p))
        self._user = (C.c_void_p * 1)(C.cast(C.pointer(self.sub), C.c_void_p))

    def run(self, ticks: int, window: int = 1):
        """Returns (binds, seconds); raises KsError (with the binds before it) as Run would."""
        out = (_lib.KsBind * max(ticks, 1))()
        n = C.c_int64(0)
        sec = C.c_double(0)
        rc = self.L.ks_run(self.eng.h, ticks, window, 1, self._fn, self._user, out, ticks, C.byref(n), C.byref(sec))
        arr = np.frombuffer(out, dtype=np.dtype([("pod", "<i8"), ("node", "<i4"), ("status", "<i4"),
                                                 ("tick", "<i8")]), count=min(n.value, ticks)).copy()
        self.eng._submitted = int(self.sub.next)
        if rc != _lib.KS_OK:
            raise KsError(rc, self.eng._L.ks_last_error(self.eng.h).decode(), arr)
        return arr, sec.value


def head_probe(eng: Engine, tick: int):
    """The Go adapters' per-pod work on the queue's head: ``Device.Filter`` / ``Device.Score``
    (go/kubesim/engine/plugins.go) over ``ks_filter`` / ``ks_score``."""
    total = eng._submitted
    q = total - eng.queued
    if eng.queued > 0:
        eng.filter(q)
        eng.score(q)


def timed(fn, *a, **kw):
    t0 = time.perf_counter()
    fn(*a, **kw)
    return time.perf_counter() - t0
