"""the device path on a label/taint domain past one 64-bit mask per node — 50k
nodes, each with a unique ``kubernetes.io/hostname`` label, 130 distinct taints (120
NoSchedule/NoExecute; tracegen.wide_trace) — encoded by kubesim_amd.encode (referenced label pairs,
toleration classes of taints) and scheduled bind-for-bind against the oracle, which filters on the
strings themselves (oracle/ks_oracle.c: ToleratesTaint, nodeSelector pairs).  The same
cluster also goes through the C++ ingest as config text (ks_cluster_parse_ex, ks_cluster_note_pod,
ks_cluster_seal; tests/harness.py cluster_yaml)."""
import numpy as np
import pytest

from harness import assert_same_binds, encoded, engine_run, ingest_encoded, make_engine, make_oracle
from kubesim_amd import _lib, encode, tracegen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wide():
    tr = tracegen.wide_trace(n_nodes=50_000, n_pods=12_000)
    enc = encoded(tr)
    assert len(np.unique(tr["nodes"]["label"], axis=0)) > 50_000   # unique hostnames
    assert len(enc["label_dict"]) <= encode.MAX_LABEL_BITS and len(enc["taint_dict"]) <= encode.MAX_TAINT_BITS
    ora = make_oracle(tr, "feeds_all_lrba")
    ora.set_threads(8)
    ora.submit(tr)
    ob, rc = ora.step(tr["pods"]["m"], cap=tr["pods"]["m"])
    return tr, enc, ob, rc


@pytest.mark.parametrize("flags", [0, _lib.KS_ENGINE_NO_OVERLAP], ids=["chunk_overlap", "plain_chain"])
def test_wide_domain_matches_oracle(wide, flags):
    tr, enc, ob, rc = wide
    eng = make_engine(tr, enc, "feeds_all_lrba", engine_flags=flags)
    eng.submit(enc["pods"])
    eb, erc = engine_run(eng, tr["pods"]["m"], 4096)
    assert erc == rc
    assert_same_binds(eb, ob)
    # the hostname-selecting pods landed on their one node
    hs = np.nonzero(np.diff(tr["pods"]["sel_off"]) == 1)[0]
    assert len(hs) > 0


def test_wide_domain_through_cpp_ingest_matches_oracle(wide):
    tr, _enc, ob, rc = wide
    enc, c = ingest_encoded(tr)
    assert c.n == 50_000
    eng = make_engine(tr, enc, "feeds_all_lrba")
    eng.submit(enc["pods"])
    eb, erc = engine_run(eng, tr["pods"]["m"], 4096)
    assert erc == rc
    assert_same_binds(eb, ob)
