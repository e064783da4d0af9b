"""Host ingest: the bitmask encodings must decide taint/toleration and nodeSelector exactly as
the literal string predicates do (toleration.go:37-56; PodSpec.NodeSelector, types.go:2805)."""
import numpy as np
import pytest

from harness import small_trace
from kubesim_amd import encode, tracegen
from pysim import PySim


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_masks_match_literal_predicates(seed):
    tr = small_trace(seed, n_nodes=60, n_pods=120, bad_selector_p=0.05)
    enc = encode.encode_trace(tr)
    ps = PySim(tr)
    ps.submit(tr)
    p = enc["pods"]
    for j in range(tr["pods"]["m"]):
        pod = ps.pods[j]
        for n in range(tr["nodes"]["n"]):
            taint_ok = (int(enc["taint"][n]) & ~int(p["tol"][j]) & 0xFFFFFFFFFFFFFFFF) == 0
            sel_ok = (int(enc["label"][n]) & int(p["sel"][j])) == int(p["sel"][j])
            assert taint_ok == ps._taint_ok(n, pod), (j, n)
            assert sel_ok == ps._selector_ok(n, pod), (j, n)


def test_tolerates_truth_table():
    E, NS, PNS, NE = tracegen.EFFECT_NONE, tracegen.NO_SCHEDULE, tracegen.PREFER_NO_SCHEDULE, tracegen.NO_EXECUTE
    EQ, EX, BAD = tracegen.OP_EQUAL, tracegen.OP_EXISTS, tracegen.OP_INVALID
    key, val = 5, 7
    cases = [
        # (tol key, op, tol value, tol effect) -> tolerates taint (5, 7, NoSchedule)?
        ((5, EQ, 7, NS), True), ((5, EQ, 7, E), True), ((5, EQ, 8, NS), False),
        ((5, EX, 0, E), True), ((6, EX, 0, E), False), ((0, EX, 0, E), True),
        ((0, EX, 0, NE), False), ((5, EQ, 7, NE), False), ((5, BAD, 7, NS), False),
        ((0, EQ, 7, E), True),   # empty key matches all keys; Equal still compares values
        ((0, EQ, 0, E), False),
    ]
    for (k, op, v, e), want in cases:
        got = bool(encode.tolerates(np.array([k]), np.array([op]), np.array([v]), np.array([e]), key, val, NS)[0])
        assert got == want, ((k, op, v, e), want)
        lit = PySim._tolerates(dict(key="k" if k else "", op={0: "Equal", 1: "Exists", 2: "X"}[op],
                                    value={7: "v7", 8: "v8", 0: ""}[v],
                                    effect={0: "", 1: "NoSchedule", 3: "NoExecute"}[e]),
                               ("k" if k == 5 else "other", "v7", "NoSchedule"))
        if k in (0, 5):
            assert lit == want


def test_absent_keys_and_pods_capacity():
    tr = tracegen.c1_trace(4)
    tr["nodes"]["alloc_has"] = np.array([15 & ~4, 15 & ~8], dtype=np.uint8)
    enc = encode.encode_trace(tr)
    assert enc["alloc"][0, tracegen.GPU] == -1          # absent gpu key ⇒ -1
    assert enc["alloc"][1, tracegen.PODS] == 0          # absent pods ⇒ Pods().Value() == 0


def test_negative_inputs_rejected():
    tr = tracegen.c1_trace(2)
    tr["pods"]["req"][0, 0] = -1
    with pytest.raises(encode.EncodeError):
        encode.encode_trace(tr)


@pytest.mark.parametrize("seed", [0, 1])
def test_wide_domain_masks_match_literal_predicates(seed):
    """a cluster past one 64-bit mask — a unique hostname label per node (more
    than 63 label pairs) and 130 distinct taints (120 NoSchedule/NoExecute) — encodes referenced
    label pairs only and one bit per toleration class of taints, and still decides every (pod, node)
    exactly as the literal string predicates do."""
    tr = tracegen.wide_trace(n_nodes=800, n_pods=90, seed=0x77 + seed, host_sel_permille=80)
    assert len(np.unique(tr["nodes"]["label"], axis=0)) > encode.MAX_LABEL_BITS
    t = tr["nodes"]["taint"]
    assert len(np.unique(t[t[:, 2] != tracegen.PREFER_NO_SCHEDULE], axis=0)) > encode.MAX_TAINT_BITS
    enc = encode.encode_trace(tr)
    assert len(enc["label_dict"]) <= encode.MAX_LABEL_BITS and len(enc["taint_dict"]) <= encode.MAX_TAINT_BITS
    ps = PySim(tr)
    ps.submit(tr)
    p = enc["pods"]
    hosts = 0
    for j in range(tr["pods"]["m"]):
        pod = ps.pods[j]
        for n in range(tr["nodes"]["n"]):
            taint_ok = (int(enc["taint"][n]) & ~int(p["tol"][j]) & 0xFFFFFFFFFFFFFFFF) == 0
            sel_ok = (int(enc["label"][n]) & int(p["sel"][j])) == int(p["sel"][j])
            assert taint_ok == ps._taint_ok(n, pod), (j, n)
            assert sel_ok == ps._selector_ok(n, pod), (j, n)
            hosts += sel_ok and p["sel"][j] != 0 and bin(int(p["sel"][j])).count("1") == 1
    assert hosts > 0


def test_wide_domain_full_size_encodes():
    """The 50k-node form of the wide trace (unique hostnames, 130 taints) fits one mask per node."""
    tr = tracegen.wide_trace()
    enc = encode.encode_trace(tr)
    assert tr["nodes"]["n"] == 50_000
    assert len(enc["taint_dict"]) <= encode.MAX_TAINT_BITS and len(enc["label_dict"]) <= encode.MAX_LABEL_BITS
