"""Host ingest: structured trace → the int64 SoA + bitmask records the C-ABI takes.

This is the host half of the Filter predicates of SURVEY.md §8(a13):

* taints: the distinct ``(key, value, effect)`` triples with effect NoSchedule or
  NoExecute are dictionary-encoded; a node carries the OR of its taints' bits.
  PreferNoSchedule never filters, so it gets no bit.  For every pod the host evaluates
  ``Toleration.ToleratesTaint`` (``vendor/k8s.io/api/core/v1/toleration.go:37-56``) of each
  of its tolerations against every dictionary taint, once, and ships the OR as ``tol``.
  The device test is then ``(node_taint & ~tol) == 0``.
* labels: the distinct ``(key, value)`` node-label pairs are dictionary-encoded; a pod's
  nodeSelector becomes ``sel``; a selector pair no node carries sets bit 63, which no node
  ever has, so the pod is infeasible everywhere.  Device test: ``(label & sel) == sel``.
* capacity: ``alloc[n][4]`` in milli-units for cpu / memory / gpu with ``-1`` for an absent
  key (absent fails every requested key, ``kubesim/node/resource.go:54-55``), and
  ``Capacity.Pods().Value()`` (absent ⇒ 0, ``vendor/k8s.io/api/core/v1/resource.go:44-49``).
* requests: ``req[m][3]`` plus a key-presence mask (``getResourceReq``,
  ``kubesim/node/resource.go:43-49``).

Inputs must be non-negative; the device's incremental admission relies on it.
"""
from __future__ import annotations

import numpy as np

from .tracegen import (CPU, GPU, MEM, NO_EXECUTE, NO_SCHEDULE, OP_EQUAL, OP_EXISTS, PODS,
                       EFFECT_NONE)

SEL_IMPOSSIBLE = np.uint64(1) << np.uint64(63)
MAX_TAINT_BITS = 64
MAX_LABEL_BITS = 63


class EncodeError(ValueError):
    """Raised for inputs outside the device path's exact domain (maps to KS_EINVAL)."""


def _or_reduce_csr(bits: np.ndarray, off: np.ndarray) -> np.ndarray:
    n = len(off) - 1
    out = np.zeros(n, dtype=np.uint64)
    if len(bits) == 0:
        return out
    counts = np.diff(off)
    nz = counts > 0
    red = np.bitwise_or.reduceat(bits, off[:-1][nz].astype(np.int64))
    out[nz] = red
    return out


def _unique_rows(rows: np.ndarray):
    """Sorted distinct rows of a small non-negative int table and each row's index into them.

    Rows are packed into one int64 key when the columns fit (lexicographic order is kept),
    which is much faster than ``np.unique(axis=0)`` on millions of rows."""
    rows = rows.astype(np.int64)
    ncol = rows.shape[1]
    bits = 63 // ncol
    if rows.min() >= 0 and rows.max() < (1 << bits):
        key = np.zeros(len(rows), dtype=np.int64)
        for c in range(ncol):
            key = (key << bits) | rows[:, c]
        uk, inv = np.unique(key, return_inverse=True)
        mask = (1 << bits) - 1
        uniq = np.stack([(uk >> (bits * (ncol - 1 - c))) & mask for c in range(ncol)], axis=1)
        return uniq, inv.reshape(-1)
    uniq, inv = np.unique(rows, axis=0, return_inverse=True)
    return uniq, inv.reshape(-1)


def _taint_classes(uniq, pods):
    """Wide taint domains (> 64 distinct NoSchedule/NoExecute taints): taints that exactly the same
    pods tolerate are interchangeable for the filter — a node is feasible for pod p iff p tolerates
    every one of its taints — so one bit per class of equal toleration signatures (over every pod of
    the trace, ``Toleration.ToleratesTaint`` as ``tolerates``) decides exactly as one bit per taint.
    Returns each taint's class and the classes' representatives (a pod tolerates a class iff it
    tolerates its representative)."""
    tol = pods["tol"]
    sig_class, cls, reps = {}, np.zeros(len(uniq), dtype=np.int64), []
    for i, (k, v, e) in enumerate(uniq):
        if len(tol):
            hit = tolerates(tol[:, 0], tol[:, 1], tol[:, 2], tol[:, 3], int(k), int(v), int(e)).astype(np.uint64)
            per_pod = _or_reduce_csr(hit, pods["tol_off"]) != 0
        else:
            per_pod = np.zeros(pods["m"], dtype=bool)
        key = np.packbits(per_pod).tobytes()
        if key not in sig_class:
            sig_class[key] = len(reps)
            reps.append(tuple(int(x) for x in (k, v, e)))
        cls[i] = sig_class[key]
    return cls, reps


def encode_nodes(nodes: dict, pods: dict | None = None):
    """Return ``(alloc[n][4] i64, taint[n] u64, label[n] u64, taint_dict, label_dict)``.

    With the trace's ``pods`` the domain widens where one 64-bit mask per node
    would not hold it: more than 63 distinct label pairs encode only the pairs some pod's
    nodeSelector references (no other label can change a placement — per-node hostname labels
    need no bits), and more than 64 distinct NoSchedule/NoExecute taints encode one bit per class of
    taints that the same pods tolerate (``_taint_classes``).  Within one mask the encoding is the
    plain one-bit-per-entry dictionary."""
    n = nodes["n"]
    alloc = nodes["alloc"].astype(np.int64).copy()
    has = nodes["alloc_has"]
    if (alloc < 0).any():
        raise EncodeError("negative capacity is outside the device path's domain")
    for k, bit in ((CPU, 1), (MEM, 2), (GPU, 4)):
        alloc[(has & bit) == 0, k] = -1
    alloc[(has & 8) == 0, PODS] = 0

    t = nodes["taint"]
    filt = (t[:, 2] == NO_SCHEDULE) | (t[:, 2] == NO_EXECUTE) if len(t) else np.zeros(0, bool)
    tbits = np.zeros(len(t), dtype=np.uint64)
    taint_dict = []
    if filt.any():
        # sorted distinct rows: the order of sorted(set(tuples)).
        uniq, inv = _unique_rows(t[filt])
        taint_dict = [tuple(int(x) for x in r) for r in uniq]
        bit_of = np.arange(len(taint_dict), dtype=np.int64)
        if len(taint_dict) > MAX_TAINT_BITS and pods is not None:
            bit_of, taint_dict = _taint_classes(uniq, pods)
        if len(taint_dict) > MAX_TAINT_BITS:
            raise EncodeError(f"{len(taint_dict)} distinct NoSchedule/NoExecute taint classes > {MAX_TAINT_BITS} (W=1)")
        tbits[filt] = np.left_shift(np.uint64(1), bit_of[inv.reshape(-1)].astype(np.uint64))
    node_taint = _or_reduce_csr(tbits, nodes["taint_off"])

    lab = nodes["label"]
    pairs = []
    lbits = np.zeros(len(lab), dtype=np.uint64)
    if len(lab):
        uniq, inv = _unique_rows(lab)
        pairs = [(int(r[0]), int(r[1])) for r in uniq]
        keep = np.ones(len(pairs), dtype=bool)
        if len(pairs) > MAX_LABEL_BITS and pods is not None:  # only the pairs a selector references
            sel = pods["sel"]
            ref = set(zip(sel[:, 0].tolist(), sel[:, 1].tolist())) if len(sel) else set()
            keep = np.array([pr in ref for pr in pairs], dtype=bool)
            pairs = [pr for pr, k in zip(pairs, keep) if k]
        if len(pairs) > MAX_LABEL_BITS:
            raise EncodeError(f"{len(pairs)} distinct (referenced) label pairs > {MAX_LABEL_BITS} (W=1)")
        bit = np.cumsum(keep) - 1
        lbits = np.where(keep[inv.reshape(-1)], np.left_shift(np.uint64(1), np.maximum(bit[inv.reshape(-1)], 0).astype(np.uint64)),
                         np.uint64(0)).astype(np.uint64)
    node_label = _or_reduce_csr(lbits, nodes["label_off"])
    assert n == len(alloc)
    return alloc, node_taint, node_label, taint_dict, pairs


def tolerates(tkey, top, tval, teff, key, val, eff):
    """Vectorised ``Toleration.ToleratesTaint`` (toleration.go:37-56); id 0 = empty string."""
    ok = (teff == EFFECT_NONE) | (teff == eff)
    ok &= (tkey == 0) | (tkey == key)
    ok &= ((top == OP_EQUAL) & (tval == val)) | (top == OP_EXISTS)
    return ok


def encode_pods(pods: dict, taint_dict, label_dict):
    """Return the per-pod device records (dict of arrays) for ``ks_submit_pods``."""
    m = pods["m"]
    req = pods["req"].astype(np.int64)
    if (req < 0).any():
        raise EncodeError("negative request is outside the device path's domain")
    if (pods["phase_use"] < 0).any():
        raise EncodeError("negative usage is outside the device path's domain")
    keymask = pods["req_has"].astype(np.uint8) & 7
    req = np.where(((keymask[:, None] >> np.arange(3)) & 1) == 1, req, 0)

    tol = pods["tol"]
    rowbits = np.zeros(len(tol), dtype=np.uint64)
    if len(tol):
        for i, (k, v, e) in enumerate(taint_dict):
            hit = tolerates(tol[:, 0], tol[:, 1], tol[:, 2], tol[:, 3], int(k), int(v), int(e))
            rowbits |= np.where(hit, np.uint64(1) << np.uint64(i), np.uint64(0))
    tolmask = _or_reduce_csr(rowbits, pods["tol_off"])

    sel = pods["sel"]
    sbits = np.zeros(len(sel), dtype=np.uint64)
    if len(sel):
        keys = (sel[:, 0].astype(np.int64) << 32) | sel[:, 1].astype(np.int64)
        lut = {(int(k) << 32) | int(v): i for i, (k, v) in enumerate(label_dict)}
        uniq, inv = np.unique(keys, return_inverse=True)
        ubits = np.array([np.uint64(1) << np.uint64(lut[int(u)]) if int(u) in lut else SEL_IMPOSSIBLE
                          for u in uniq], dtype=np.uint64)
        sbits = ubits[inv]
    selmask = _or_reduce_csr(sbits, pods["sel_off"])

    use = pods["phase_use"].astype(np.int64)
    phas = pods["phase_has"].astype(np.uint8)
    use = np.where(((phas[:, None] >> np.arange(3)) & 1) == 1, use, 0)
    return dict(m=m, arrival=pods["arrival"].astype(np.int64), req=np.ascontiguousarray(req),
                keymask=keymask, tol=tolmask, sel=selmask,
                phase_off=pods["phase_off"].astype(np.int32),
                phase_sec=pods["phase_sec"].astype(np.int32),
                phase_use=np.ascontiguousarray(use), flags=pods["flags"].astype(np.uint8),
                key_id=np.asarray(pods["key_id"], dtype=np.int64) if "key_id" in pods else None)


def encode_trace(trace: dict):
    alloc, taint, label, tdict, ldict = encode_nodes(trace["nodes"], trace["pods"])
    pods = encode_pods(trace["pods"], tdict, ldict)
    return dict(alloc=alloc, taint=taint, label=label, taint_dict=tdict, label_dict=ldict, pods=pods)
