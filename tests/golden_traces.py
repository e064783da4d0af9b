"""Seeded small traces whose expected binds / usage are committed in tests/golden/.

The fixture stores only the generator parameters and the expected outputs; the trace itself
is regenerated (tracegen is deterministic).  Expected outputs were produced by the C oracle
and cross-checked against the independent Python restatement (tests/golden/make_golden.py).
"""
from __future__ import annotations

import hashlib

import numpy as np

from harness import MODES

CASES = [
    dict(name="c3like_feeds", seed=101, n_nodes=512, n_pods=300, mode="feeds_all_lrba", ticks=320,
         kw=dict(taints=True, labels=True, tolerations=True, selectors=True, arrival="stream")),
    dict(name="c2like_literal", seed=102, n_nodes=40, n_pods=400, mode="literal_lrba_filters_ignored",
         ticks=420, kw=dict(taints=False, labels=False, tolerations=False, selectors=False, arrival="bulk")),
    dict(name="c2like_feeds_fit", seed=103, n_nodes=16, n_pods=500, mode="feeds_fit_lr", ticks=520,
         kw=dict(taints=False, labels=False, tolerations=False, selectors=False, arrival="bulk", short=True)),
    dict(name="taint_sel_const", seed=104, n_nodes=256, n_pods=200, mode="feeds_taint_sel_ba_const",
         ticks=260, kw=dict(taints=True, labels=True, tolerations=True, selectors=True, arrival="stream",
                            bad_selector_p=0.01)),
]


def build_trace(case):
    from kubesim_amd import tracegen
    kw = dict(case["kw"])
    short = kw.pop("short", False)
    tr = tracegen.synth_trace(case["n_nodes"], case["n_pods"], case["seed"], **kw)
    if short:
        ps = tr["pods"]["phase_sec"]
        ps[:] = 3 + (np.arange(len(ps)) * 7919) % 300
    return tr


def usage_digest(u):
    return hashlib.sha256(np.ascontiguousarray(u, dtype=np.int64).tobytes()).hexdigest()[:16]


def run_oracle(case):
    from pyoracle import COracle
    fm, fl, sc = MODES[case["mode"]]
    tr = build_trace(case)
    co = COracle(tr, filter_mode=fm, filters=fl, scorers=sc)
    co.submit(tr)
    binds, usage, rc = [], [], 0
    for _ in range(case["ticks"]):
        b, rc = co.step(1)
        binds += [[int(b["pod"][i]), int(b["node"][i]), int(b["tick"][i]), int(b["status"][i])]
                  for i in range(len(b["pod"]))]
        if rc:
            break
        usage.append(usage_digest(co.usage()))
    return dict(binds=binds, usage=usage, rc=int(rc), tick=int(co.tick))


def run_engine(case):
    from harness import encoded, make_engine
    from kubesim_amd.engine import KsError
    tr = build_trace(case)
    enc = encoded(tr)
    eng = make_engine(tr, enc, case["mode"])
    eng.submit(enc["pods"])
    binds, usage, rc = [], [], 0
    for _ in range(case["ticks"]):
        try:
            b = eng.step(1)
        except KsError as e:
            b, rc = e.binds, e.code
        binds += [[int(x["pod"]), int(x["node"]), int(x["tick"]), int(x["status"])] for x in b]
        if rc:
            break
        usage.append(usage_digest(eng.usage()))
    return dict(binds=binds, usage=usage, rc=int(rc), tick=int(eng.tick))


def check_case(case_gold, who):
    case = next(c for c in CASES if c["name"] == case_gold["name"])
    got = run_oracle(case) if who == "oracle" else run_engine(case)
    assert got["rc"] == case_gold["rc"], (case["name"], got["rc"], case_gold["rc"])
    assert got["tick"] == case_gold["tick"], case["name"]
    assert got["binds"] == case_gold["binds"], case["name"]
    assert got["usage"] == case_gold["usage"], case["name"]
