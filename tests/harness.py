"""Shared parity harness: run the HIP engine and the CPU oracle on the same trace."""
from __future__ import annotations

import numpy as np

from kubesim_amd import encode, tracegen
from pyoracle import COracle

# (filter_mode, filters, scorers) combinations exercised by the parity suites
MODES = {
    "literal_const": (0, 0, ((0, 1, 1),)),
    "literal_lrba_filters_ignored": (0, 7, ((1, 1, 0), (2, 1, 0))),
    "feeds_all_lrba": (1, 7, ((1, 1, 0), (2, 1, 0))),
    "feeds_fit_lr": (1, 1, ((1, 2, 0),)),
    "feeds_taint_sel_ba_const": (1, 6, ((2, 3, 0), (0, 2, 5))),
    "no_scorers": (1, 7, ()),
}


def make_engine(trace, enc, mode, batch_pods=0, engine_flags=0, shard=None):
    """shard = (world, rank, comm_id, vshards) for a node-sharded engine (Engine.shard)."""
    from kubesim_amd.engine import Engine
    fm, fl, sc = MODES[mode] if isinstance(mode, str) else mode
    eng = Engine(tick_seconds=trace["tick_seconds"], filter_mode=fm, filters=fl, scorers=sc,
                 batch_pods=batch_pods, engine_flags=engine_flags)
    if shard is not None:
        eng.shard(*shard)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    return eng


def make_oracle(trace, mode):
    fm, fl, sc = MODES[mode] if isinstance(mode, str) else mode
    return COracle(trace, filter_mode=fm, filters=fl, scorers=sc)


def engine_run(eng, ticks, chunk):
    """Step the engine in chunks; returns (binds array, error code or 0)."""
    from kubesim_amd.engine import KsError
    out = []
    left = ticks
    while left > 0:
        k = min(chunk, left)
        try:
            out.append(eng.step(k))
        except KsError as e:
            out.append(e.binds)
            return np.concatenate(out), e.code
        left -= k
    return (np.concatenate(out) if out else np.zeros(0)), 0


def oracle_run(ora, ticks):
    b, rc = ora.step(ticks, cap=ticks)
    return b, rc


def assert_same_binds(eb, ob):
    assert len(eb) == len(ob["pod"]), (len(eb), len(ob["pod"]))
    np.testing.assert_array_equal(eb["pod"], ob["pod"])
    np.testing.assert_array_equal(eb["tick"], ob["tick"])
    bad = np.nonzero((eb["node"] != ob["node"]) | (eb["status"] != ob["status"]))[0]
    assert len(bad) == 0, f"first mismatch at bind {bad[0]}: engine {eb[bad[0]]} oracle " \
                          f"node {ob['node'][bad[0]]} status {ob['status'][bad[0]]}"


def small_trace(seed, n_nodes=24, n_pods=200, **kw):
    kw.setdefault("taints", True)
    kw.setdefault("labels", True)
    kw.setdefault("tolerations", True)
    kw.setdefault("selectors", True)
    return tracegen.synth_trace(n_nodes, n_pods, seed, **kw)


def encoded(trace):
    return encode.encode_trace(trace)


_EFF = {1: "NoSchedule", 2: "PreferNoSchedule", 3: "NoExecute"}
_TOL_EFF = {0: "", 1: "NoSchedule", 2: "PreferNoSchedule", 3: "NoExecute"}
_OPS = {0: "Equal", 1: "Exists", 2: "Bogus"}


def cluster_yaml(trace):
    """A trace's nodes as the reference's cluster config text (kubesim/config/config.go:15-41):
    quantities in milli-units, taints and labels as strings, nodes named node-i."""
    from kubesim_amd import tracegen
    st, nd = trace["strings"], trace["nodes"]
    out = [f"tick: {trace['tick_seconds']}", "cluster:", "  nodes:"]
    names = (("cpu", tracegen.HAS_CPU), ("memory", tracegen.HAS_MEM), ("nvidia.com/gpu", tracegen.HAS_GPU))
    q = lambda s: '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'
    for i in range(nd["n"]):
        has = int(nd["alloc_has"][i])
        out += [f"  - namespace: default", f"    name: node-{i}", "    capacity:"]
        for k, (nm, bit) in enumerate(names):
            if has & bit:
                out.append(f"      {nm}: {int(nd['alloc'][i, k])}m")
        if has & tracegen.HAS_PODS:
            out.append(f"      pods: {int(nd['alloc'][i, tracegen.PODS])}")
        a, b = nd["taint_off"][i], nd["taint_off"][i + 1]
        if b > a:
            out.append("    taints:")
            for k, v, e in nd["taint"][a:b]:
                out += [f"    - key: {q(st[k])}", f"      value: {q(st[v])}", f"      effect: {_EFF[int(e)]}"]
        a, b = nd["label_off"][i], nd["label_off"][i + 1]
        if b > a:
            out.append("    labels:")
            out += [f"      {q(st[k])}: {q(st[v])}" for k, v in nd["label"][a:b]]
    return "\n".join(out) + "\n"


def pod_strings(trace):
    """Each pod's (tolerations, nodeSelector pairs) as the strings ks_cluster_* take."""
    st, p = trace["strings"], trace["pods"]
    out = []
    for q in range(p["m"]):
        a, b = p["tol_off"][q], p["tol_off"][q + 1]
        tols = [(st[k], _OPS[int(o)], st[v], _TOL_EFF[int(e)]) for k, o, v, e in p["tol"][a:b]]
        a, b = p["sel_off"][q], p["sel_off"][q + 1]
        out.append((tols, [(st[k], st[v]) for k, v in p["sel"][a:b]]))
    return out


def ingest_encoded(trace):
    """encode.encode_trace's output with the cluster and the pods' masks taken through the C++
    ingest instead (ks_cluster_parse_ex / ks_cluster_note_pod / ks_cluster_seal when the cluster is
    past one mask, ks_cluster_tolerations / ks_cluster_selector per pod)."""
    from kubesim_amd.ingest import Cluster
    ps = pod_strings(trace)
    c = Cluster(cluster_yaml(trace), pods=ps)
    enc = encode.encode_trace(trace)
    pods = dict(enc["pods"])
    pods["tol"] = np.array([c.tolerations(t) for t, _ in ps], dtype=np.uint64)
    pods["sel"] = np.array([c.selector(s) for _, s in ps], dtype=np.uint64)
    np.testing.assert_array_equal(c.alloc, enc["alloc"])
    return dict(alloc=c.alloc, taint=c.taint, label=c.label, pods=pods), c
