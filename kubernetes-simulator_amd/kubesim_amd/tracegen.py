"""Seeded synthetic cluster + pod-trace generator (SURVEY.md §8(d) configs C1–C5).

The reference has no trace format of its own: pods come from an ``api.Submitter``
(``api/submitter.go:10-16``; the example one is ``examples/main.go:79-137``) and nodes from
the YAML config (``kubesim/config/config.go:15-41``).  This module produces the same
*information* in a structured, string-interned form:

* nodes: capacity (milli-units for cpu / memory / nvidia.com/gpu, plain count for
  ``pods``) with per-key presence, taints ``(key, value, effect)``
  (``vendor/k8s.io/api/core/v1/types.go:2660-2674``), labels ``(key, value)``;
* pods: arrival tick (the tick whose ``Submit`` call returns the pod), container-summed
  requests with per-key presence (``kubesim/node/resource.go:43-49``), tolerations
  ``(key, operator, value, effect)`` (``types.go:2701-2726``), nodeSelector pairs
  (``types.go:2805``) and the simSpec phases (``kubesim/pod/spec.go:16-19``).

Strings are interned; id 0 is always the empty string so ``len(t.Key) > 0`` in
``toleration.go:42`` becomes ``key != 0``.

Everything is generated with counter-based splitmix64 so any element can be regenerated
from ``(seed, stream, index)`` and the output is identical on every machine.
All quantities are integers in milli-units, which is exact for every value generated
(``resource.Quantity`` semantics, ``quantity.go:30-99``).
"""
from __future__ import annotations

import numpy as np

GI = 1 << 30
MI = 1 << 20
MILLI = 1000

# resource slot order used everywhere in this repo
CPU, MEM, GPU, PODS = 0, 1, 2, 3
HAS_CPU, HAS_MEM, HAS_GPU, HAS_PODS = 1, 2, 4, 8

# taint / toleration effects (types.go:2683-2696); 0 = empty (toleration only)
EFFECT_NONE, NO_SCHEDULE, PREFER_NO_SCHEDULE, NO_EXECUTE = 0, 1, 2, 3
# toleration operators (types.go:2728-2733); anything else never tolerates (toleration.go:53)
OP_EQUAL, OP_EXISTS, OP_INVALID = 0, 1, 2

_U64 = np.uint64
_GOLDEN = _U64(0x9E3779B97F4A7C15)


def splitmix64(x):
    """splitmix64 finaliser over a uint64 array (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = (x + _GOLDEN).astype(np.uint64)
        z = (z ^ (z >> _U64(30))) * _U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U64(27))) * _U64(0x94D049BB133111EB)
        return z ^ (z >> _U64(31))


def draw(seed: int, stream: int, idx) -> np.ndarray:
    """Counter-based random u64 for element ``idx`` of ``stream``."""
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = splitmix64(np.array([(seed ^ (stream * 0xD1B54A32D192ED03)) & 0xFFFFFFFFFFFFFFFF],
                                   dtype=np.uint64))[0]
        return splitmix64(base + idx * _GOLDEN)


def uniform_int(seed, stream, idx, k):
    return (draw(seed, stream, idx) % _U64(k)).astype(np.int64)


class StringTable:
    def __init__(self):
        self.strings = [""]
        self.index = {"": 0}

    def intern(self, s: str) -> int:
        i = self.index.get(s)
        if i is None:
            i = len(self.strings)
            self.strings.append(s)
            self.index[s] = i
        return i


def _csr_from_counts(counts):
    off = np.zeros(len(counts) + 1, dtype=np.int32)
    np.cumsum(counts, out=off[1:])
    return off


# ---------------------------------------------------------------------------------------------
# C1: config/sample.yml + examples/main.go
# ---------------------------------------------------------------------------------------------

def c1_trace(n_pods: int = 1000):
    """The reference's own runnable case (BASELINE.json configs[0]).

    Nodes from ``config/sample.yml:16-35``; pod ``n`` is returned by the example submitter
    at the (n+1)-th tick (``examples/main.go:84-85``: ``elapsed/5 >= n`` with a 10 s tick);
    requests ``{cpu 3, memory 5Gi, nvidia.com/gpu 1}`` (``:116-120``), simSpec phases
    ``5 s {1, 2Gi, 0}`` then ``10 s {2, 4Gi, 1}`` (``:96-107``).
    """
    st = StringTable()
    k_os, v_sim = st.intern("beta.kubernetes.io/os"), st.intern("simulated")
    nodes = dict(
        n=2,
        names=["node-0", "node-1"],
        alloc=np.array([[4 * MILLI, 8 * GI * MILLI, 1 * MILLI, 2],
                        [8 * MILLI, 16 * GI * MILLI, 2 * MILLI, 4]], dtype=np.int64),
        alloc_has=np.array([15, 15], dtype=np.uint8),
        taint_off=np.zeros(3, dtype=np.int32), taint=np.zeros((0, 3), dtype=np.int32),
        label_off=np.array([0, 1, 2], dtype=np.int32),
        label=np.array([[k_os, v_sim], [k_os, v_sim]], dtype=np.int32),
    )
    m = n_pods
    pods = dict(
        m=m,
        arrival=np.arange(1, m + 1, dtype=np.int64),
        req=np.tile(np.array([3 * MILLI, 5 * GI * MILLI, 1 * MILLI], dtype=np.int64), (m, 1)),
        req_has=np.full(m, 7, dtype=np.uint8),
        tol_off=np.zeros(m + 1, dtype=np.int32), tol=np.zeros((0, 4), dtype=np.int32),
        sel_off=np.zeros(m + 1, dtype=np.int32), sel=np.zeros((0, 2), dtype=np.int32),
        phase_off=np.arange(0, 2 * m + 1, 2, dtype=np.int32),
        phase_sec=np.tile(np.array([5, 10], dtype=np.int32), m),
        phase_use=np.tile(np.array([[1 * MILLI, 2 * GI * MILLI, 0],
                                    [2 * MILLI, 4 * GI * MILLI, 1 * MILLI]], dtype=np.int64), (m, 1)),
        phase_has=np.full(2 * m, 7, dtype=np.uint8),
        key_id=np.arange(m, dtype=np.int64),
        flags=np.zeros(m, dtype=np.uint8),
    )
    return dict(config="C1", tick_seconds=10, strings=st.strings, nodes=nodes, pods=pods)


# ---------------------------------------------------------------------------------------------
# C2 / C3 / C4 / C5 synthetic clusters
# ---------------------------------------------------------------------------------------------

CPU_CHOICES = np.array([8, 16, 32, 64, 128], dtype=np.int64) * MILLI
MEM_CHOICES = np.array([32, 64, 128, 256, 512], dtype=np.int64) * GI * MILLI
GPU_CHOICES = np.array([0, 0, 2, 4, 8], dtype=np.int64) * MILLI

ZONES, TYPES, GPUTYPES = 8, 16, 4
LABEL_KEYS = ["topology.kubernetes.io/zone", "node.kubernetes.io/instance-type",
              "accelerator/gpu-type", "kubernetes.io/os"]
LABEL_CARD = [ZONES, TYPES, GPUTYPES, 1]
N_TAINTS = 16


def _taint_dict(st: StringTable):
    """16 dictionary taints: 8 NoSchedule, 4 NoExecute, 4 PreferNoSchedule (§8(d) C3)."""
    out = []
    for j in range(N_TAINTS):
        eff = NO_SCHEDULE if j < 8 else (NO_EXECUTE if j < 12 else PREFER_NO_SCHEDULE)
        out.append((st.intern(f"taint.sim/k{j % 10}"), st.intern(f"v{j % 3}"), eff))
    return np.array(out, dtype=np.int32)


def _label_value(st, fam, v):
    if fam == 0:
        return st.intern(f"zone-{v}")
    if fam == 1:
        return st.intern(f"type-{v}")
    if fam == 2:
        return st.intern(f"gpu-{v}")
    return st.intern("linux" if v == 0 else f"os-{v}")


def synth_trace(n_nodes: int, n_pods: int, seed: int, *, taints: bool, labels: bool,
                tolerations: bool, selectors: bool, arrival: str = "bulk",
                bad_selector_p: float = 0.0, gpu_absent_p: float = 0.05,
                node_offset: int = 0, config: str = "synthetic", max_sel_pairs: int = 2,
                mem_decimal: bool = False):
    """Generate a synthetic trace with the §8(d) distributions.

    ``arrival="bulk"`` makes every pod arrive at tick 1 (a Submitter returning the whole
    trace on its first call); ``"stream"`` spaces arrivals 0–2 ticks apart so the FIFO
    sometimes runs empty (``kubesim/kubesim.go:144-147``).
    ``node_offset`` shifts node-indexed draws so a shard of a bigger cluster can be
    generated without materialising the whole cluster.
    ``mem_decimal``: memory requests in decimal SI (``500M`` .. ``32G`` in 500M steps) on the
    binary-SI capacities (``32Gi`` .. ``512Gi``) — the common real-world mix: the gcd of the
    memory quantities drops to 2^8 bytes and the capacities scale to 2^31, outside the engine's
    32-bit evaluators (the wide class).
    """
    st = StringTable()
    N, P = int(n_nodes), int(n_pods)
    nid = np.arange(N, dtype=np.uint64) + np.uint64(node_offset)

    alloc = np.zeros((N, 4), dtype=np.int64)
    alloc[:, CPU] = CPU_CHOICES[uniform_int(seed, 1, nid, 5)]
    alloc[:, MEM] = MEM_CHOICES[uniform_int(seed, 2, nid, 5)]
    alloc[:, GPU] = GPU_CHOICES[uniform_int(seed, 3, nid, 5)]
    alloc[:, PODS] = 110
    gpu_absent = (uniform_int(seed, 4, nid, 1_000_000) < int(gpu_absent_p * 1_000_000))
    alloc_has = np.where(gpu_absent, HAS_CPU | HAS_MEM | HAS_PODS, 15).astype(np.uint8)
    alloc[gpu_absent, GPU] = 0

    tdict = _taint_dict(st)
    if taints:
        u = uniform_int(seed, 5, nid, 10)
        ntaint = np.where(u < 8, 0, 1 + uniform_int(seed, 6, nid, 2)).astype(np.int32)
        t_off = _csr_from_counts(ntaint)
        first = uniform_int(seed, 7, nid, N_TAINTS)
        second = (first + 1 + uniform_int(seed, 8, nid, N_TAINTS - 1)) % N_TAINTS
        rows = np.zeros((int(t_off[-1]), 3), dtype=np.int32)
        owner = np.repeat(np.arange(N), ntaint)
        slot = np.arange(int(t_off[-1])) - t_off[owner]
        pick = np.where(slot == 0, first[owner], second[owner])
        rows[:] = tdict[pick]
    else:
        t_off = np.zeros(N + 1, dtype=np.int32)
        rows = np.zeros((0, 3), dtype=np.int32)

    if labels:
        lkeys = [st.intern(k) for k in LABEL_KEYS]
        lvals = [[_label_value(st, f, v) for v in range(LABEL_CARD[f])] for f in range(4)]
        lab = np.zeros((N, 4, 2), dtype=np.int32)
        for f in range(4):
            v = uniform_int(seed, 9 + f, nid, LABEL_CARD[f])
            lab[:, f, 0] = lkeys[f]
            lab[:, f, 1] = np.array(lvals[f], dtype=np.int32)[v]
        l_off = np.arange(0, 4 * N + 1, 4, dtype=np.int32)
        lrows = lab.reshape(-1, 2)
    else:
        l_off = np.zeros(N + 1, dtype=np.int32)
        lrows = np.zeros((0, 2), dtype=np.int32)

    nodes = dict(n=N, alloc=alloc, alloc_has=alloc_has, taint_off=t_off, taint=rows,
                 label_off=l_off, label=lrows)

    # ---------------- pods ----------------
    pid = np.arange(P, dtype=np.uint64)
    if arrival == "bulk":
        arr = np.ones(P, dtype=np.int64)
    elif arrival == "stream":
        gaps = uniform_int(seed, 20, pid, 3)  # 0,1,2 ticks between arrivals
        arr = 1 + np.cumsum(gaps)
    else:
        raise ValueError(arrival)
    req = np.zeros((P, 3), dtype=np.int64)
    req[:, CPU] = (1 + uniform_int(seed, 21, pid, 80)) * 100
    if mem_decimal:
        req[:, MEM] = (1 + uniform_int(seed, 22, pid, 64)) * 500_000_000 * MILLI
    else:
        req[:, MEM] = (1 + uniform_int(seed, 22, pid, 128)) * 256 * MI * MILLI
    gsel = uniform_int(seed, 23, pid, 10)
    req[:, GPU] = np.where(gsel < 7, 0, np.array([1, 2, 4], dtype=np.int64)[uniform_int(seed, 24, pid, 3)] * MILLI)
    req_has = np.full(P, 7, dtype=np.uint8)

    nph = (1 + uniform_int(seed, 25, pid, 4)).astype(np.int32)
    p_off = _csr_from_counts(nph)
    F = int(p_off[-1])
    fid = np.arange(F, dtype=np.uint64)
    owner = np.repeat(np.arange(P), nph)
    p_sec = (10 + uniform_int(seed, 26, fid, 36000 - 10 + 1)).astype(np.int32)
    pct = np.array([25, 50, 75, 100], dtype=np.int64)[uniform_int(seed, 27, fid, 4)]
    p_use = req[owner] * pct[:, None] // 100
    p_has = np.full(F, 7, dtype=np.uint8)

    if tolerations:
        ntol = uniform_int(seed, 30, pid, 4).astype(np.int32)
        tl_off = _csr_from_counts(ntol)
        K = int(tl_off[-1])
        kid = np.arange(K, dtype=np.uint64)
        kind = uniform_int(seed, 31, kid, 16)
        j = uniform_int(seed, 32, kid, N_TAINTS)
        vrand = np.array([st.intern(f"v{x}") for x in range(4)], dtype=np.int32)[uniform_int(seed, 33, kid, 4)]
        tk = tdict[j, 0]
        tv = tdict[j, 1]
        te = tdict[j, 2]
        tol = np.zeros((K, 4), dtype=np.int32)
        # kind 0: empty key + Exists, any effect (tolerates everything)
        # kind 1: empty key + Exists + NoSchedule
        # 2..7: Equal, exact taint j; 8..11: Exists key j, empty effect
        # 12..14: Equal key j with a random value, empty effect; 15: invalid operator
        key = np.where(kind <= 1, 0, tk)
        op = np.where(kind <= 1, OP_EXISTS,
                      np.where((kind >= 8) & (kind <= 11), OP_EXISTS,
                               np.where(kind == 15, OP_INVALID, OP_EQUAL)))
        val = np.where(kind <= 1, 0, np.where((kind >= 8) & (kind <= 11), 0,
                                              np.where((kind >= 12) & (kind <= 14), vrand, tv)))
        eff = np.where(kind == 0, EFFECT_NONE, np.where(kind == 1, NO_SCHEDULE,
                       np.where((kind >= 2) & (kind <= 7), te, EFFECT_NONE)))
        # keep "tolerate everything" rare: only 1 of 4 kind-0 draws stays kind 0
        rare = uniform_int(seed, 34, kid, 4) != 0
        demote = (kind == 0) & rare
        key = np.where(demote, tk, key)
        op = np.where(demote, OP_EQUAL, op)
        val = np.where(demote, tv, val)
        eff = np.where(demote, te, eff)
        tol[:, 0], tol[:, 1], tol[:, 2], tol[:, 3] = key, op, val, eff
    else:
        tl_off = np.zeros(P + 1, dtype=np.int32)
        tol = np.zeros((0, 4), dtype=np.int32)

    if selectors and labels:
        has_sel = uniform_int(seed, 40, pid, 10) < 3
        nsel = np.where(has_sel, 1 + uniform_int(seed, 41, pid, max_sel_pairs), 0).astype(np.int32)
        s_off = _csr_from_counts(nsel)
        S = int(s_off[-1])
        sid = np.arange(S, dtype=np.uint64)
        sowner = np.repeat(np.arange(P), nsel)
        slot = np.arange(S) - s_off[sowner]
        fam0 = uniform_int(seed, 42, pid, 4)
        fam1 = (fam0 + 1 + uniform_int(seed, 43, pid, 3)) % 4
        fam = np.where(slot == 0, fam0[sowner], fam1[sowner])
        card = np.array(LABEL_CARD, dtype=np.int64)[fam]
        v = (draw(seed, 44, sid) % card.astype(np.uint64)).astype(np.int64)
        lkeys = np.array([st.intern(k) for k in LABEL_KEYS], dtype=np.int32)
        vals = np.zeros(S, dtype=np.int32)
        for f in range(4):
            table = np.array([_label_value(st, f, x) for x in range(LABEL_CARD[f])], dtype=np.int32)
            mf = fam == f
            vals[mf] = table[v[mf]]
        if bad_selector_p > 0:
            bad = uniform_int(seed, 45, sid, 1_000_000) < int(bad_selector_p * 1_000_000)
            vals[bad & (fam == 0)] = st.intern("zone-nowhere")
        sel = np.stack([lkeys[fam], vals], axis=1).astype(np.int32)
    else:
        s_off = np.zeros(P + 1, dtype=np.int32)
        sel = np.zeros((0, 2), dtype=np.int32)

    pods = dict(m=P, arrival=arr, req=req, req_has=req_has, tol_off=tl_off, tol=tol,
                sel_off=s_off, sel=sel, phase_off=p_off, phase_sec=p_sec, phase_use=p_use,
                phase_has=p_has, key_id=np.arange(P, dtype=np.int64),
                flags=np.zeros(P, dtype=np.uint8))
    return dict(config=config, tick_seconds=10, strings=st.strings, nodes=nodes, pods=pods)


def wide_trace(n_nodes=50_000, n_pods=20_000, seed=0x5EED0006, n_taint_keys=30, n_taint_vals=4, n_host_sel=24,
               host_sel_permille=2):
    """A cluster past one 64-bit mask per node: every node carries a unique
    ``kubernetes.io/hostname`` label beside the C3 families, and the taint dictionary holds
    ``n_taint_keys`` x ``n_taint_vals`` NoSchedule / NoExecute taints (120 by default) plus 10
    PreferNoSchedule.  A quarter of the nodes carry one or two of them.  Pods tolerate with the C3
    mix of kinds, but their keys come from the first ten taint keys only (clusters carry more taints
    than any pod tolerates); ``host_sel_permille`` / 1000 of the pods select the hostname of one of ``n_host_sel`` untainted
    nodes (and nothing else; 100m CPU, 128Mi, no GPU), the rest select C3 families as ``c3_trace`` does."""
    tr = synth_trace(n_nodes, n_pods, seed, taints=False, labels=True, tolerations=False, selectors=True,
                     config="wide")
    st = StringTable()
    st.strings = list(tr["strings"])
    st.index = {x: i for i, x in enumerate(st.strings)}
    N, P = int(n_nodes), int(n_pods)
    nid = np.arange(N, dtype=np.uint64)
    pid = np.arange(P, dtype=np.uint64)
    # taints
    T = n_taint_keys * n_taint_vals
    tdict = []
    for j in range(T):
        eff = NO_EXECUTE if j % 3 == 2 else NO_SCHEDULE
        tdict.append((st.intern(f"taint.wide/k{j % n_taint_keys}"), st.intern(f"w{j // n_taint_keys}"), eff))
    for j in range(10):
        tdict.append((st.intern(f"taint.wide/pref{j}"), st.intern("x"), PREFER_NO_SCHEDULE))
    tdict = np.array(tdict, dtype=np.int32)
    u = uniform_int(seed, 50, nid, 4)
    ntaint = np.where(u < 3, 0, 1 + uniform_int(seed, 51, nid, 2)).astype(np.int32)
    t_off = _csr_from_counts(ntaint)
    first = uniform_int(seed, 52, nid, len(tdict))
    second = (first + 1 + uniform_int(seed, 53, nid, len(tdict) - 1)) % len(tdict)
    owner = np.repeat(np.arange(N), ntaint)
    slot = np.arange(int(t_off[-1])) - t_off[owner]
    rows = tdict[np.where(slot == 0, first[owner], second[owner])].astype(np.int32)
    nodes = tr["nodes"]
    nodes["taint_off"], nodes["taint"] = t_off, rows
    # a unique hostname label per node (after the four families)
    host_key = st.intern("kubernetes.io/hostname")
    lab = nodes["label"].reshape(N, 4, 2)
    host = np.array([[host_key, st.intern(f"node-{i:07d}")] for i in range(N)], dtype=np.int32)
    nodes["label"] = np.concatenate([lab, host[:, None, :]], axis=1).reshape(-1, 2)
    nodes["label_off"] = np.arange(0, 5 * N + 1, 5, dtype=np.int32)
    # tolerations over the first ten taint keys (the C3 kinds)
    ntol = uniform_int(seed, 54, pid, 4).astype(np.int32)
    tl_off = _csr_from_counts(ntol)
    K = int(tl_off[-1])
    kid = np.arange(K, dtype=np.uint64)
    kind = uniform_int(seed, 55, kid, 16)
    j = uniform_int(seed, 56, kid, 10) + n_taint_keys * uniform_int(seed, 57, kid, n_taint_vals)
    tk, tv, te = tdict[j, 0], tdict[j, 1], tdict[j, 2]
    vrand = np.array([st.intern(f"w{x}") for x in range(n_taint_vals + 1)], dtype=np.int32)[
        uniform_int(seed, 58, kid, n_taint_vals + 1)]
    rare = uniform_int(seed, 59, kid, 4) != 0
    kind = np.where((kind == 0) & rare, 2, kind)
    key = np.where(kind <= 1, 0, tk)
    op = np.where(kind <= 1, OP_EXISTS, np.where((kind >= 8) & (kind <= 11), OP_EXISTS,
                                                  np.where(kind == 15, OP_INVALID, OP_EQUAL)))
    val = np.where(kind <= 1, 0, np.where((kind >= 8) & (kind <= 11), 0,
                                          np.where((kind >= 12) & (kind <= 14), vrand, tv)))
    eff = np.where(kind == 0, EFFECT_NONE, np.where(kind == 1, NO_SCHEDULE,
                   np.where((kind >= 2) & (kind <= 7), te, EFFECT_NONE)))
    pods = tr["pods"]
    pods["tol_off"] = tl_off
    pods["tol"] = np.stack([key, op, val, eff], axis=1).astype(np.int32)
    # 0.2 % of the pods: a hostname selector alone (one of n_host_sel untainted nodes)
    untainted = np.nonzero((ntaint == 0) & (nodes["alloc_has"] == 15))[0]
    hosts = untainted[(np.arange(n_host_sel) * 7919) % len(untainted)]
    hsel = uniform_int(seed, 60, pid, 1000) < host_sel_permille
    pick = hosts[uniform_int(seed, 61, pid, n_host_sel)]
    s_off, sel = pods["sel_off"], pods["sel"]
    nsel = np.diff(s_off)
    nsel = np.where(hsel, 1, nsel).astype(np.int32)
    new_off = _csr_from_counts(nsel)
    new_sel = np.zeros((int(new_off[-1]), 2), dtype=np.int32)
    for i in np.nonzero(~hsel & (np.diff(s_off) > 0))[0]:
        new_sel[new_off[i]:new_off[i + 1]] = sel[s_off[i]:s_off[i + 1]]
    hi = np.nonzero(hsel)[0]
    new_sel[new_off[hi], 0] = host_key
    new_sel[new_off[hi], 1] = host[pick[hi], 1]
    pods["sel_off"], pods["sel"] = new_off, new_sel
    pods["req"][hsel] = (100, 128 * 2**20 * MILLI, 0)   # a pinned pod is small: its node must keep room
    tr["strings"] = st.strings
    return tr


def c2_trace(n_nodes=5000, n_pods=100_000, seed=0x5EED0002, **kw):
    """BASELINE.json configs[1]: 5k nodes / 100k pods, cpu+mem+gpu, multi-phase simSpec."""
    return synth_trace(n_nodes, n_pods, seed, taints=False, labels=False, tolerations=False,
                       selectors=False, config="C2", **kw)


def c3_trace(n_nodes=50_000, n_pods=1_000_000, seed=0x5EED0003, **kw):
    """BASELINE.json configs[2]: 50k nodes with taints/labels, tolerations, 1M pods."""
    return synth_trace(n_nodes, n_pods, seed, taints=True, labels=True, tolerations=True,
                       selectors=True, config="C3", **kw)


def c3q_trace(n_nodes=50_000, n_pods=1_000_000, seed=0x5EED0003, **kw):
    """C3 with realistic quantities: decimal-SI memory requests (500M, 1G,
    3G, ...) on binary-SI capacities (64Gi .. 512Gi), as resource.Quantity accepts any mix
    (vendor/k8s.io/apimachinery/pkg/api/resource/quantity.go:531-566)."""
    kw.setdefault("mem_decimal", True)
    return synth_trace(n_nodes, n_pods, seed, taints=True, labels=True, tolerations=True,
                       selectors=True, config="C3q", **kw)


def c4_scenario(s: int, n_nodes=2000, n_pods=10_000, **kw):
    """BASELINE.json configs[3]: scenario ``s`` of 1024 independent what-if clusters.

    C3 distributions, except that a nodeSelector names one label pair: with two pairs on a
    2k-node cluster some pod matches no node within the first few thousand pods of every
    scenario (checked with the oracle: 24 of 24 seeds), and the run stops with NotFound exactly
    as the reference's would (kubesim/kubesim.go:217-220) — a degenerate what-if workload."""
    kw.setdefault("max_sel_pairs", 1)
    return synth_trace(n_nodes, n_pods, 0x5EED0004 ^ s, taints=True, labels=True,
                       tolerations=True, selectors=True, config=f"C4[{s}]", **kw)


def c5_trace(n_nodes=1 << 20, n_pods=100_000, seed=0x5EED0005, **kw):
    """BASELINE.json configs[4]: 1M nodes (8 × 131,072), 100k pods."""
    return synth_trace(n_nodes, n_pods, seed, taints=True, labels=True, tolerations=True,
                       selectors=True, config="C5", **kw)


def slice_pods(trace, lo, hi):
    """Return a copy of ``trace`` keeping pods ``[lo, hi)`` (CSR re-based)."""
    p = trace["pods"]
    out = dict(m=hi - lo, arrival=p["arrival"][lo:hi].copy(), req=p["req"][lo:hi].copy(),
               req_has=p["req_has"][lo:hi].copy(), key_id=p["key_id"][lo:hi].copy(),
               flags=p["flags"][lo:hi].copy())
    for name, cols in (("tol", None), ("sel", None), ("phase", None)):
        off = p[f"{name}_off"]
        a, b = int(off[lo]), int(off[hi])
        out[f"{name}_off"] = (off[lo:hi + 1] - a).astype(np.int32)
        if name == "phase":
            out["phase_sec"] = p["phase_sec"][a:b].copy()
            out["phase_use"] = p["phase_use"][a:b].copy()
            out["phase_has"] = p["phase_has"][a:b].copy()
        else:
            out[name] = p[name][a:b].copy()
    t = dict(trace)
    t["pods"] = out
    return t
