"""Python handle over the C-ABI (include/ks_engine.h): the device scheduling engine.

``Engine`` mirrors the reference's engine surface (kubesim/kubesim.go):

=====================  ==============================================================
reference              here
=====================  ==============================================================
NewKubeSim             ``Engine(tick_seconds, filter_mode, filters, scorers)`` +
                       ``load_nodes`` (kubesim/kubesim.go:32-61)
RegisterFilter /       ``filters`` bits / ``scorers`` list, fixed at creation
RegisterScorer         (kubesim/kubesim.go:78-86); built-in device plugins only
submit (Submitter)     ``submit`` (kubesim/kubesim.go:126-139)
Run                    ``step(ticks)`` — advances the tick loop (kubesim/kubesim.go:90-123)
api.Filter / Scorer    ``filter(pod)`` / ``score(pod)``
=====================  ==============================================================

Errors come back as :class:`KsError` with the reference's kind (``InvalidArgument`` /
``NotFound``); binds made before an aborting error are still returned by ``step``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import KsBind, KsConfig, KsStepStats


class KsError(RuntimeError):
    def __init__(self, code: int, msg: str, binds=None):
        super().__init__(f"{_lib.STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code
        self.kind = _lib.STATUS_NAMES.get(code, str(code))
        self.binds = binds


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def _config(tick_seconds, filter_mode, filters, scorers, device, batch_pods, engine_flags):
    cfg = KsConfig()
    cfg.abi_version = _lib.KS_ABI_VERSION
    cfg.tick_seconds = tick_seconds
    cfg.filter_mode = filter_mode
    cfg.filters = filters
    cfg.n_scorers = len(scorers)
    for i, (k, w, v) in enumerate(scorers):
        cfg.scorers[i].kind, cfg.scorers[i].weight, cfg.scorers[i].value = k, w, v
    cfg.device = device
    cfg.batch_pods = batch_pods
    cfg.engine_flags = engine_flags
    return cfg


class Engine:
    def __init__(self, *, tick_seconds=10, filter_mode=_lib.KS_FILTER_REFERENCE_LITERAL, filters=0,
                 scorers=((_lib.KS_SCORER_CONST, 1, 1),), device=0, batch_pods=0, engine_flags=0,
                 _group=None):
        L = _lib.load()
        self._group = _group
        cfg = _config(tick_seconds, filter_mode, filters, scorers, device, batch_pods, engine_flags)
        h = C.c_void_p()
        if _group is None:
            rc = L.ks_create(C.byref(cfg), C.byref(h))
        else:
            rc = L.ks_group_add(_group.h, C.byref(cfg), C.byref(h))
        if rc != _lib.KS_OK:
            raise KsError(rc, "ks_create / ks_group_add rejected the configuration")
        self._L = L
        self.h = h
        self.n = 0
        self._submitted = 0

    def close(self):
        if getattr(self, "h", None):
            if getattr(self, "_group", None) is None:  # a group's members die with the group
                self._L.ks_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc, binds=None):
        if rc != _lib.KS_OK:
            raise KsError(rc, self._L.ks_last_error(self.h).decode(), binds)

    # -- node sharding ------------------------------------------------------
    def shard(self, world: int, rank: int, comm_id: bytes | None = None, vshards: int = 1):
        """Scan only this rank's node range; candidates are all-gathered per batch over RCCL
        (comm_id from :func:`comm_unique_id` on rank 0, broadcast by the caller).  Before
        ``load_nodes``.  ``vshards`` > 1 splits the range further (one-GPU testing)."""
        buf = None
        if comm_id is not None:
            if len(comm_id) != _lib.KS_COMM_ID_BYTES:
                raise ValueError("comm_id must be KS_COMM_ID_BYTES long")
            buf = (C.c_uint8 * _lib.KS_COMM_ID_BYTES).from_buffer_copy(comm_id)
        self._check(self._L.ks_shard(self.h, world, rank, buf, vshards))

    def shard_host(self, world: int, rank: int, exchange: "LocalExchange", vshards: int = 1):
        """Node sharding with a host exchange instead of RCCL (ks_shard_host): ranks are engines
        driven by threads of this process, exchanging candidates through ``exchange``."""
        self._xchg = exchange  # keep alive
        self._check(self._L.ks_shard_host(self.h, world, rank, vshards, exchange.fn, exchange.h))

    # -- cluster / queue ---------------------------------------------------------------------
    def load_nodes(self, alloc, taint, label):
        alloc = _c(alloc, np.int64).reshape(-1, 4)
        self.n = len(alloc)
        self._check(self._L.ks_load_nodes(self.h, self.n, _p(alloc), _p(_c(taint, np.uint64)),
                                          _p(_c(label, np.uint64))))

    def submit(self, pods: dict):
        """Append encoded pods (see kubesim_amd.encode.encode_pods).  ``key_id`` (optional,
        int64 per pod): interned namespace-name keys; absent/None = every pod its own key."""
        m = int(pods["m"])
        arrs = [_c(pods["arrival"], np.int64), _c(pods["req"], np.int64).reshape(-1, 3),
                _c(pods["keymask"], np.uint8), _c(pods["tol"], np.uint64), _c(pods["sel"], np.uint64),
                _c(pods["phase_off"], np.int32), _c(pods["phase_sec"], np.int32),
                _c(pods["phase_use"], np.int64).reshape(-1, 3), _c(pods["flags"], np.uint8)]
        keys = pods.get("key_id")
        if keys is not None:
            keys = _c(keys, np.int64)
        # the C side reads these lengths blindly: check them here
        per_pod = {"arrival": arrs[0], "req": arrs[1], "keymask": arrs[2], "tol": arrs[3], "sel": arrs[4],
                   "flags": arrs[8]}
        if keys is not None:
            per_pod["key_id"] = keys
        for name, a in per_pod.items():
            if len(a) != m:
                raise ValueError(f"pods[{name!r}] has {len(a)} rows, expected m = {m}")
        off = arrs[5]
        if len(off) != m + 1:
            raise ValueError(f"pods['phase_off'] has {len(off)} entries, expected m + 1 = {m + 1}")
        nf = int(off[-1]) if m else 0
        if m and (off[0] != 0 or (np.diff(off) < 0).any()):
            raise ValueError("pods['phase_off'] must start at 0 and be non-decreasing")
        if len(arrs[6]) < nf or len(arrs[7]) < nf:
            raise ValueError(f"phase arrays shorter than phase_off[-1] = {nf}")
        ptrs = [_p(a) for a in arrs] + [_p(keys) if keys is not None else None]
        self._check(self._L.ks_submit_pods(self.h, m, *ptrs))
        self._submitted += m

    # -- tick loop ---------------------------------------------------------------------------
    def step(self, ticks: int, cap: int | None = None):
        """Advance ``ticks`` ticks; returns binds as a structured numpy array
        (pod, node, status, tick).  ``cap`` defaults to the binds the step can make (at most one
        per tick and one per queued pod)."""
        if cap is None:
            cap = max(0, min(ticks, self.queued))
        out = (KsBind * max(cap, 1))()
        n = C.c_int64(0)
        rc = self._L.ks_step(self.h, ticks, out, cap, C.byref(n))
        k = min(n.value, cap)
        arr = np.frombuffer(out, dtype=np.dtype([("pod", "<i8"), ("node", "<i4"), ("status", "<i4"),
                                                 ("tick", "<i8")]), count=k).copy()
        self._check(rc, arr)
        return arr

    def filter(self, pod: int):
        mask = np.zeros(self.n, np.uint8)
        self._check(self._L.ks_filter(self.h, pod, _p(mask)))
        return mask

    def score(self, pod: int):
        score = np.zeros(self.n, np.int64)
        self._check(self._L.ks_score(self.h, pod, _p(score)))
        return score

    def usage(self):
        out = np.zeros((self.n, 3), np.int64)
        self._check(self._L.ks_usage(self.h, _p(out)))
        return out

    def usage_at(self, t: int):
        """Per-node usage [n][3] at any past tick 0 <= t <= the current tick."""
        out = np.zeros((self.n, 3), np.int64)
        self._check(self._L.ks_usage_at(self.h, t, _p(out)))
        return out

    def usage_digest(self, t_lo: int, t_hi: int):
        """[t_hi - t_lo][6] uint64: per tick Σ_n usage[n][k] (k < 3) and Σ_n mix(n) usage[n][k-3]."""
        out = np.zeros((max(t_hi - t_lo, 0), 6), np.uint64)
        self._check(self._L.ks_usage_digest(self.h, t_lo, t_hi, _p(out)))
        return out

    def pod_lookup(self, node: int, key_id: int):
        """Node.GetPod: FIFO index of the pod stored on ``node`` under ``key_id`` (KsError NotFound)."""
        q = C.c_int64(-1)
        self._check(self._L.ks_pod_lookup(self.h, node, key_id, C.byref(q)))
        return q.value

    def node_pods(self, node: int):
        """Node.GetPodList: FIFO indices of the pods stored on ``node`` (one per key)."""
        n = C.c_int64(0)
        self._check(self._L.ks_node_pods(self.h, node, None, 0, C.byref(n)))
        out = np.zeros(max(n.value, 1), np.int64)
        self._check(self._L.ks_node_pods(self.h, node, _p(out), n.value, C.byref(n)))
        return out[:n.value].copy()

    def pod_status(self, pod_lo: int = 0, n: int | None = None):
        """Pod.BuildStatus phases (kubesim/pod/pod.go:78-145) at the current tick: structured
        array (phase, node, start_tick, total_seconds); phases _lib.KS_PHASE_*."""
        n = (self._submitted - pod_lo) if n is None else n
        out = (_lib.KsPodInfo * max(n, 1))()
        self._check(self._L.ks_pod_status(self.h, pod_lo, n, out))
        dt = np.dtype([("phase", "<i4"), ("node", "<i4"), ("start_tick", "<i8"), ("total_seconds", "<i4"),
                       ("pad", "<i4")])
        return np.frombuffer(out, dtype=dt, count=n).copy()

    @property
    def tick(self):
        return self._L.ks_current_tick(self.h)

    @property
    def queued(self):
        return self._L.ks_queued_pods(self.h)

    def last_step_stats(self):
        s = KsStepStats()
        self._L.ks_last_step_stats(self.h, C.byref(s))
        return dict(step_ms=s.step_ms, scan_ms=s.scan_ms, resolve_ms=s.resolve_ms, launches=s.launches,
                    pods=s.pods, other_ms=s.other_ms)

    def last_step_kernels(self):
        """Per-kernel event times of the last profiled step (include/ks_engine.h ks_kernel_stats)."""
        s = _lib.KsKernelStats()
        self._check(self._L.ks_last_step_kernels(self.h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in s._fields_}

    def debug_counters(self):
        out = np.zeros(32, np.int64)
        self._check(self._L.ks_debug_counters(self.h, _p(out)))
        return out

    def debug_invariants(self):
        """Between-step invariants (include/ks_engine.h ks_debug_invariants): slot marks left set,
        E-index marks left set (both must be 0), the most candidate slots a batch claimed, the staged
        slots."""
        out = np.zeros(4, np.int64)
        self._check(self._L.ks_debug_invariants(self.h, _p(out)))
        return dict(slot_marks=int(out[0]), e_marks=int(out[1]), nslot_hw=int(out[2]), slot_max=int(out[3]))

    def debug_window(self) -> bytes:
        """The raw batch window workspace (include/ks_engine.h ks_debug_window; diagnostics)."""
        n = C.c_int64(0)
        self._check(self._L.ks_debug_window(self.h, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        self._check(self._L.ks_debug_window(self.h, buf, n.value, C.byref(n)))
        return buf.raw

    def debug_watch(self, pod: int):
        """Record pod's batch in the window workspace (a -DKS_BATCH_LOG diagnostic build only)."""
        self._check(self._L.ks_debug_watch(self.h, pod))

    def set_profiling(self, on: bool):
        self._L.ks_set_profiling(self.h, 1 if on else 0)


def engine_for_trace(trace, enc, **cfg):
    """Create an Engine loaded with an encoded trace's nodes."""
    eng = Engine(tick_seconds=trace["tick_seconds"], **cfg)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    return eng


def selftest(test: int = _lib.KS_SELFTEST_LR_MICRO, device: int = 0) -> int:
    """Run a device self-test (include/ks_engine.h, ks_selftest); returns the failure count."""
    L = _lib.load()
    n = C.c_int64(-1)
    rc = L.ks_selftest(device, test, C.byref(n))
    if rc != 0:
        raise KsError(rc, "ks_selftest failed")
    return n.value


class LocalExchange:
    """An in-process all-gather for ``world`` engines sharded with :meth:`Engine.shard_host`
    (ks_local_allgather, include/ks_kubesim.h)."""

    def __init__(self, world: int):
        self._R = _lib.load_run()
        self.h = self._R.ks_local_exchange_create(world)
        if not self.h:
            raise ValueError("bad world size")
        self.fn = C.cast(self._R.ks_local_allgather, C.c_void_p)

    def abort(self):
        """End every current and later exchange with KS_EDEVICE (a rank failed before its
        deposit: the others would wait for it forever; ks_local_exchange_abort)."""
        if getattr(self, "h", None):
            self._R.ks_local_exchange_abort(self.h)

    def close(self):
        if getattr(self, "h", None):
            self._R.ks_local_exchange_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


def comm_unique_id() -> bytes:
    """A fresh RCCL communicator id for :meth:`Engine.shard` (create on rank 0 only)."""
    L = _lib.load()
    buf = (C.c_uint8 * _lib.KS_COMM_ID_BYTES)()
    rc = L.ks_comm_unique_id(buf)
    if rc != 0:
        raise KsError(rc, "ks_comm_unique_id failed")
    return bytes(buf)


class Group:
    """Independent what-if scenarios (BASELINE.json configs[3]) stepped together on one device:
    one launch per kernel for all members (include/ks_engine.h, ks_group_*)."""

    def __init__(self, max_scenarios: int, device: int = 0):
        self._L = _lib.load()
        h = C.c_void_p()
        rc = self._L.ks_group_create(device, max_scenarios, C.byref(h))
        if rc != _lib.KS_OK:
            raise KsError(rc, "ks_group_create failed")
        self.h = h
        self.device = device
        self.members = []

    def add(self, **cfg) -> Engine:
        """A member engine (same keyword configuration as :class:`Engine`)."""
        cfg.setdefault("device", self.device)
        e = Engine(_group=self, **cfg)
        self.members.append(e)
        return e

    def step(self, ticks: int, cap: int | None = None):
        """Advance every member ``ticks`` ticks.  Returns (binds, counts, statuses, stats):
        ``binds`` is one structured array (pod, node, status, tick) holding member i's binds at
        rows [i * cap, i * cap + counts[i]) — :meth:`split` cuts it per member."""
        S = len(self.members)
        if cap is None:  # at most one bind per tick and per queued pod of the longest queue
            cap = max(0, min(ticks, max((e.queued for e in self.members), default=0)))
        if getattr(self, "_out_n", -1) < S * cap:  # reused across steps (no per-step 10s of MB)
            self._out = (KsBind * max(S * cap, 1))()
            self._out_n = S * cap
        n = np.zeros(S, np.int64)
        st = np.zeros(S, np.int32)
        stats = KsStepStats()
        rc = self._L.ks_group_step(self.h, ticks, self._out, cap, _p(n), _p(st), C.byref(stats))
        if rc != _lib.KS_OK:
            raise KsError(rc, "ks_group_step failed")
        dt = np.dtype([("pod", "<i8"), ("node", "<i4"), ("status", "<i4"), ("tick", "<i8")])
        allb = np.frombuffer(self._out, dtype=dt, count=S * cap) if S * cap else np.zeros(0, dt)
        self._cap = cap
        return allb, np.minimum(n, cap), st, dict(step_ms=stats.step_ms, launches=stats.launches, pods=stats.pods)

    def split(self, binds, counts):
        """Per-member copies of the binds returned by :meth:`step`."""
        return [binds[i * self._cap:i * self._cap + int(c)].copy() for i, c in enumerate(counts)]

    def close(self):
        if getattr(self, "h", None):
            for e in self.members:
                e.h = None
            self._L.ks_group_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()
