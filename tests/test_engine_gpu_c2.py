"""GPU parity over the whole of BASELINE.json configs[1] (C2: 5,000 nodes, 100,000 pods, cpu +
memory + nvidia.com/gpu requests, multi-phase simSpec), in both filter modes.

The oracle finishes C2 in seconds (OpenMP over nodes), so this is an exact bind-for-bind and
usage-for-usage comparison of the full run, not a prefix: every pod's node, status and tick,
and every node's per-tick usage at the chunk boundaries (kubesim/kubesim.go:90-225,
kubesim/node/node.go:36-60, kubesim/pod/pod.go:47-69).
"""
import numpy as np
import pytest

from harness import assert_same_binds, encoded, engine_run, make_engine, make_oracle, oracle_run
from kubesim_amd import tracegen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c2():
    tr = tracegen.c2_trace()
    return tr, encoded(tr)


@pytest.mark.parametrize("mode", ["feeds_all_lrba", "literal_lrba_filters_ignored"])
def test_c2_full_run_matches_oracle(c2, mode):
    tr, enc = c2
    m = tr["pods"]["m"]
    eng = make_engine(tr, enc, mode)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.set_threads(8)
    ora.submit(tr)
    done = 0
    for chunk in (7, 4993, 20_000, 35_000, 40_000):
        eb, erc = engine_run(eng, chunk, chunk)
        ob, orc = oracle_run(ora, chunk)
        assert erc == orc == 0
        assert_same_binds(eb, ob)
        np.testing.assert_array_equal(eng.usage(), ora.usage(), err_msg=f"usage after {done + chunk} ticks")
        done += len(eb)
    assert done == m
