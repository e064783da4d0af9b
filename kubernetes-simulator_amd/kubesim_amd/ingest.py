"""Host ingest through the C-ABI (include/ks_ingest.h): Quantity strings, the simSpec annotation,
the cluster config YAML and pod tolerations / nodeSelectors, into the engine's records.

=======================  ===================================================================
reference                here
=======================  ===================================================================
resource.ParseQuantity   ``parse_quantity`` (exact milli-units)
parseSpecYAML            ``parse_simspec`` (kubesim/pod/spec.go:35-63)
config + BuildNode       ``Cluster(yaml)`` (kubesim/config/config.go:15-110)
ToleratesTaint           ``Cluster.tolerations`` (vendor/k8s.io/api/core/v1/toleration.go:37-56)
=======================  ===================================================================
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .engine import KsError


def _cs(x):
    return x.encode() if isinstance(x, str) else x


def parse_quantity(s: str):
    """(status, milli): status KS_OK, KS_EINVAL (the reference rejects it) or KS_ERANGE (valid,
    outside the exact domain: negative, fractional milli-units, >= 2^63 milli)."""
    out = C.c_int64(0)
    rc = _lib.load().ks_parse_quantity(_cs(s), C.byref(out))
    return rc, (out.value if rc == _lib.KS_OK else None)


def parse_simspec(text: str, max_phases: int = 64):
    """[(seconds, {resource: milli})]; raises KsError (InvalidArgument / OutOfDomain)."""
    L = _lib.load()
    n = C.c_int32(0)
    sec = np.zeros(max_phases, np.int32)
    use = np.zeros((max_phases, 3), np.int64)
    mask = np.zeros(max_phases, np.uint8)
    err = C.create_string_buffer(256)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    rc = L.ks_parse_simspec(_cs(text), max_phases, C.byref(n), p(sec), p(use), p(mask), err, 256)
    if rc != _lib.KS_OK:
        raise KsError(rc, err.value.decode())
    names = ("cpu", "memory", "nvidia.com/gpu")
    return [(int(sec[i]), {names[k]: int(use[i, k]) for k in range(3) if mask[i] >> k & 1})
            for i in range(min(n.value, max_phases))]


class Cluster:
    """A parsed cluster config: node arrays for ``Engine.load_nodes`` plus the taint / label
    dictionaries pod tolerations and selectors are encoded against."""

    def __init__(self, yaml_text: str, pods=None):
        """``pods``: optional [(tolerations, selector pairs)] of every pod the cluster will see
        (``tolerations`` / ``selector`` argument forms).  Given, the masks are sealed over them
        (ks_cluster_parse_ex + ks_cluster_note_pod + ks_cluster_seal), so a cluster past one 64-bit
        mask — a hostname label per node, hundreds of taints — still encodes exactly."""
        self._L = _lib.load()
        h = C.c_void_p()
        err = C.create_string_buffer(256)
        if pods is None:
            rc = self._L.ks_cluster_parse(_cs(yaml_text), C.byref(h), err, 256)
        else:
            rc = self._L.ks_cluster_parse_ex(_cs(yaml_text), _lib.KS_CLUSTER_DEFER_MASKS, C.byref(h), err, 256)
        if rc != _lib.KS_OK:
            raise KsError(rc, err.value.decode())
        self.h = h
        if pods is not None:
            for tols, pairs in pods:
                rc = self._L.ks_cluster_note_pod(h, len(tols), *self._tol_arrays(tols), len(pairs),
                                                 *self._pair_arrays(pairs))
                if rc != _lib.KS_OK:
                    raise KsError(rc, "ks_cluster_note_pod")
            rc = self._L.ks_cluster_seal(h, err, 256)
            if rc != _lib.KS_OK:
                raise KsError(rc, err.value.decode())
        self.n = int(self._L.ks_cluster_nodes(h))
        self.tick = int(self._L.ks_cluster_tick(h))
        self.start_clock = self._L.ks_cluster_start_clock(h).decode()
        self.alloc = np.zeros((self.n, 4), np.int64)
        self.taint = np.zeros(self.n, np.uint64)
        self.label = np.zeros(self.n, np.uint64)
        p = lambda a: a.ctypes.data_as(C.c_void_p)
        self._L.ks_cluster_arrays(h, p(self.alloc), p(self.taint), p(self.label))
        self.names = [self._L.ks_cluster_node_name(h, i).decode() for i in range(self.n)]

    @staticmethod
    def _tol_arrays(tols):
        return [(C.c_char_p * max(len(tols), 1))(*[_cs(t[j] or "") for t in tols]) for j in range(4)]

    @staticmethod
    def _pair_arrays(pairs):
        return [(C.c_char_p * max(len(pairs), 1))(*[_cs(x[j]) for x in pairs]) for j in range(2)]

    def tolerations(self, tols):
        """tols: [(key, operator, value, effect)] -> tolerated-taint mask."""
        out = C.c_uint64(0)
        rc = self._L.ks_cluster_tolerations(self.h, len(tols), *self._tol_arrays(tols), C.byref(out))
        if rc != _lib.KS_OK:
            raise KsError(rc, "ks_cluster_tolerations")
        return out.value

    def selector(self, pairs):
        """pairs: [(key, value)] -> required-label mask (bit 63: a pair no node carries)."""
        out = C.c_uint64(0)
        rc = self._L.ks_cluster_selector(self.h, len(pairs), *self._pair_arrays(pairs), C.byref(out))
        if rc != _lib.KS_OK:
            raise KsError(rc, "ks_cluster_selector")
        return out.value

    def close(self):
        if getattr(self, "h", None):
            self._L.ks_cluster_free(self.h)
            self.h = None

    def __del__(self):
        self.close()
