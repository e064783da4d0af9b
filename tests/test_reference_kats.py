"""The oracle's ingest and resource-list arithmetic against the reference's own unit-test
vectors (tests/golden/reference_kats.json; sources cited there), and the C1 trace's inputs
against config/sample.yml + examples/main.go as parsed by the Quantity restatement."""
import json
import os
from datetime import datetime

import numpy as np
import pytest

import quantity as Q
from kubesim_amd import tracegen
from pysim import resource_list_ge, resource_list_sum

with open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")) as f:
    K = json.load(f)


def _milli(rl):
    return {k: Q.to_milli(v) for k, v in rl.items()}


def test_build_resource_list():
    ok, bad = K["build_resource_list"]
    assert _milli(Q.build_resource_list(ok["input"])) == ok["expect"]
    with pytest.raises(Q.QuantityError):
        Q.build_resource_list(bad["input"])


def test_parse_spec():
    ok, bad = K["parse_spec"]
    got = [[sec, _milli(rl)] for sec, rl in Q.parse_simspec(ok["input"])]
    assert got == ok["expect"]
    with pytest.raises(Q.InvalidResourceUsageField):
        Q.parse_simspec(bad["input"])


def test_resource_list_arithmetic():
    s = K["resource_list_sum"][0]
    assert resource_list_sum(s["a"], s["b"]) == s["expect"]
    assert resource_list_sum(s["b"], s["a"]) == s["expect"]
    lists = K["ge_lists"]
    for c in K["resource_list_ge"]:
        assert resource_list_ge(lists[c["a"]], lists[c["b"]]) == c["expect"], c
    d_ok, d_bad = K["resource_list_diff"]
    assert resource_list_ge(d_ok["a"], d_ok["b"])
    assert {k: v - d_ok["b"].get(k, 0) for k, v in d_ok["a"].items()} == d_ok["expect"]
    assert not resource_list_ge(d_bad["a"], d_bad["b"])


def test_taint_effects_and_clock():
    eff = {"NoSchedule": tracegen.NO_SCHEDULE, "NoExecute": tracegen.NO_EXECUTE,
           "PreferNoSchedule": tracegen.PREFER_NO_SCHEDULE}
    for c in K["build_taint"]:
        assert eff.get(c["effect"], "error") == c["expect"]
    c = K["clock_sub"]
    assert (datetime.fromisoformat(c["a"]) - datetime.fromisoformat(c["b"])).total_seconds() == c["expect_seconds"]


@pytest.mark.parametrize("s,milli", [("1", 1000), ("100m", 100), ("1.5", 1500), ("2Gi", 2 * 2**30 * 1000),
                                     ("1k", 10**6), ("1e3", 10**6), ("0", 0), ("-1", -1000), ("1n", None),
                                     ("0.5m", None), ("1Ki", 1024000), ("+2", 2000), ("Gi", 0)])
def test_quantity_units(s, milli):
    assert Q.to_milli(Q.parse_quantity(s)) == milli


@pytest.mark.parametrize("s", ["", "bar", "1Qi", "1.2.3", "1e"])
def test_quantity_invalid(s):
    with pytest.raises(Q.QuantityError):
        Q.parse_quantity(s)


def test_c1_trace_matches_reference_inputs():
    c1 = K["c1_inputs"]
    tr = tracegen.c1_trace(3)
    for i, cap in enumerate(c1["nodes"]):
        rl = Q.build_resource_list(cap)
        exp = [Q.to_milli(rl["cpu"]), Q.to_milli(rl["memory"]), Q.to_milli(rl["nvidia.com/gpu"]),
               Q.value_ceil(rl["pods"])]
        np.testing.assert_array_equal(tr["nodes"]["alloc"][i], exp)
    rq = Q.build_resource_list(c1["pod_requests"])
    np.testing.assert_array_equal(tr["pods"]["req"][0], [Q.to_milli(rq[k]) for k in ("cpu", "memory", "nvidia.com/gpu")])
    spec = Q.parse_simspec(c1["sim_spec"])
    np.testing.assert_array_equal(tr["pods"]["phase_sec"][:2], [s for s, _ in spec])
    np.testing.assert_array_equal(tr["pods"]["phase_use"][:2],
                                  [[Q.to_milli(rl[k]) for k in ("cpu", "memory", "nvidia.com/gpu")] for _, rl in spec])
    assert tr["tick_seconds"] == c1["tick"]
