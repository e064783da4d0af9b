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
