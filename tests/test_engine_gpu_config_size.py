"""GPU parity at the BASELINE.json configurations' full sizes (C3, C4).

C3 (50k nodes, 1M-pod trace, Filter fit+taint+selector -> LR+BA):
  * the first 40,000 pods bind-for-bind against the OpenMP oracle, with usage checked at sampled
    ticks of the run through ks_usage_at (the oracle stepped to each sample tick);
  * the WHOLE 1M-pod trace: the engine at the default batch and at a batch of 97 pods give
    identical binds (an exact resolver's results cannot depend on how the FIFO is cut into
    batches), plus invariants that hold for any exact implementation of the reference's loop —
    FIFO order, one bind per tick, every bind Ok under the fit filter (admission is exactly that
    predicate, kubesim/node/node.go:44-47), chosen nodes satisfy the pod's taint / selector
    filters, and the running pods' requests recomputed on the host from the binds never exceed
    any node's capacity; the per-tick usage digest agrees with ks_usage_at at sampled ticks.
  * the WHOLE trace bind-for-bind against the oracle's committed per-window digests
    (tests/golden/full_run.json) at the bench's batch, usage at every other window end;
  * the reference-literal filter mode (kubesim/kubesim.go:182: the filter result is discarded)
    on a 20,000-pod prefix against the oracle.
C4 (1024 what-if scenarios x 2,000 nodes x 10,000 pods, one group, the default batch — so the
  small-class resolver and the group-wide pods-per-workgroup are the ones exercised): EVERY
  scenario bind-for-bind and usage-for-usage against the oracle's committed digests
  (tests/golden/c4_golden.json, tests/golden/make_c4_golden.py), the aborted-scenario count
  pinned to the oracle's, every scenario checked with the invariants above.
"""
import json
import os

import numpy as np
import pytest

import full_run_digest
from harness import assert_same_binds, encoded, make_engine, make_oracle
from kubesim_amd import _lib, tracegen

pytestmark = pytest.mark.gpu
MODE = "feeds_all_lrba"
SCORERS = ((1, 1, 0), (2, 1, 0))


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS") or 0) or min(os.cpu_count() or 1, 16)


def _check_invariants(binds, first_pod, n_nodes, enc, last_tick=0):
    p = enc["pods"]
    tol = p["tol"].astype(np.uint64)
    sel = p["sel"].astype(np.uint64)
    taint = enc["taint"].astype(np.uint64)
    label = enc["label"].astype(np.uint64)
    np.testing.assert_array_equal(binds["pod"], np.arange(first_pod, first_pod + len(binds)))
    if len(binds):
        assert (np.diff(binds["tick"]) > 0).all() and binds["tick"][0] > last_tick
    assert (binds["status"] == 0).all()
    nd, q = binds["node"], binds["pod"]
    assert ((nd >= 0) & (nd < n_nodes)).all()
    assert ((taint[nd] & ~tol[q]) == 0).all()
    assert ((label[nd] & sel[q]) == sel[q]).all()


def _dur_ticks(enc, tick_seconds):
    p = enc["pods"]
    S = np.add.reduceat(p["phase_sec"].astype(np.int64), p["phase_off"][:-1]) if len(p["phase_sec"]) else 0
    S = np.where(np.diff(p["phase_off"]) > 0, S, 0)
    return np.where(S > 0, -(-S // tick_seconds), 0)


def _check_capacity(binds, enc, dur, t, n_nodes):
    """Requests of the pods running at tick t (bound Ok, t0 <= t < t0 + dur), per node, recomputed
    on the host: never above capacity, running count never above the pods capacity."""
    q, t0 = binds["pod"], binds["tick"]
    run = (t0 <= t) & (t < t0 + dur[q]) & (binds["status"] == 0)
    req = enc["pods"]["req"].reshape(-1, 3)
    alloc = enc["alloc"]
    tot = np.zeros((n_nodes, 3), np.int64)
    np.add.at(tot, binds["node"][run], req[q[run]])
    nr = np.bincount(binds["node"][run], minlength=n_nodes)
    for k in range(3):
        has = alloc[:, k] >= 0
        assert (tot[has, k] <= alloc[has, k]).all(), f"resource {k} over capacity at tick {t}"
    assert (nr <= alloc[:, 3]).all()


@pytest.fixture(scope="module")
def c3():
    tr = tracegen.c3_trace(n_nodes=50_000, n_pods=1_000_000)
    return tr, encoded(tr)


def test_c3_40k_pods_bit_exact_with_usage_samples(c3):
    tr, enc = c3
    P = 40_000
    eng = make_engine(tr, enc, MODE)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, MODE)
    ora.set_threads(_threads())
    ora.submit(tracegen.slice_pods(tr, 0, P))
    eb = eng.step(P)
    samples = (1, 977, 5000, 12_345, 25_000, P)
    obs, t = [], 0
    for s in samples:
        b, rc = ora.step(s - t, cap=s - t)
        assert rc == 0
        obs.append(b)
        t = s
        np.testing.assert_array_equal(eng.usage_at(s), ora.usage(), err_msg=f"usage at tick {s}")
    ob = {k: np.concatenate([x[k] for x in obs]) for k in obs[0]}
    assert_same_binds(eb, ob)


@pytest.mark.parametrize("batch", [160, 176, 208, 256])
def test_c3_whole_trace_at_other_batch_sizes(c3, batch):
    """The whole 1M-pod C3 trace against the oracle's digests at other batch sizes (every batch and
    chunk boundary moves: the chunk resolver's alignment-dependent stops fall on other pods)."""
    tr, enc = c3
    g = full_run_digest.load("c3")
    eng = make_engine(tr, enc, MODE, batch_pods=batch)
    eng.submit(enc["pods"])
    full_run_digest.check_engine_run(eng, g, f"c3 batch {batch}")


@pytest.mark.parametrize("flags", [0, _lib.KS_ENGINE_PRUNED_LISTS], ids=["default", "pruned_lists"])
def test_c3_whole_trace_matches_oracle_golden(c3, flags):
    """Every pod of the 1M-pod trace — the whole range bench.py times — bind-for-bind against the
    oracle's committed digests (tests/golden/full_run.json, tests/golden/make_full_run.py), at
    the bench's batch (the engine default), with usage at every other window end; the engine's
    default resolver (the chunk resolver)."""
    tr, enc = c3
    g = full_run_digest.load("c3")
    assert g is not None and g["pods"] == tr["pods"]["m"] and g["nodes"] == tr["nodes"]["n"]
    eng = make_engine(tr, enc, MODE, engine_flags=flags)
    eng.submit(enc["pods"])
    full_run_digest.check_engine_run(eng, g, "c3")


@pytest.fixture(scope="module")
def c3q():
    tr = tracegen.slice_pods(tracegen.c3q_trace(n_nodes=50_000, n_pods=1_000_000), 0, 131_072)
    return tr, encoded(tr)


@pytest.mark.parametrize("flags", [0], ids=["default"])
def test_c3q_decimal_memory_prefix_matches_oracle_golden(c3q, flags):
    """Realistic quantities: decimal-SI memory requests on binary-SI
    capacities — memory scales to 2^31 units, the wide evaluator class.  The first 131,072 pods
    bind-for-bind against the oracle's committed digests (tests/golden/full_run.json "c3q")."""
    tr, enc = c3q
    g = full_run_digest.load("c3q")
    assert g is not None and g["pods"] == tr["pods"]["m"] and g["nodes"] == tr["nodes"]["n"]
    eng = make_engine(tr, enc, MODE, engine_flags=flags)
    eng.submit(enc["pods"])
    full_run_digest.check_engine_run(eng, g, "c3q")


def test_c3_reference_literal_prefix(c3):
    """The reference's own filter behaviour at C3 size: scheduleOneFilter's result is discarded
    (kubesim/kubesim.go:182), so the filters constrain nothing and only admission decides Ok vs
    OverCapacity — 20,000 pods bind-for-bind and usage-for-usage against the oracle."""
    tr, enc = c3
    P = 20_000
    mode = "literal_lrba_filters_ignored"
    eng = make_engine(tr, enc, mode)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.set_threads(_threads())
    ora.submit(tracegen.slice_pods(tr, 0, P))
    eb = eng.step(P)
    ob, rc = ora.step(P, cap=P)
    assert rc == 0
    assert_same_binds(eb, ob)
    np.testing.assert_array_equal(eng.usage(), ora.usage())


def test_c3_whole_trace_reference_literal_matches_oracle_golden(c3):
    """The reference's own filter behaviour over the WHOLE 1M-pod C3 trace:
    scheduleOneFilter's result is discarded (kubesim/kubesim.go:182), every node is scored and only
    admission (kubesim/node/node.go:44-47) decides Ok vs OverCapacity — every window bind-for-bind
    and every other window's usage against the oracle's committed digests (tests/golden/full_run.json
    "c3lit"), at the bench's batch (bench.py's c3_literal leg)."""
    tr, enc = c3
    g = full_run_digest.load("c3lit")
    assert g is not None and g["pods"] == tr["pods"]["m"] and g["mode"] == "literal_lrba_filters_ignored"
    eng = make_engine(tr, enc, g["mode"])
    eng.submit(enc["pods"])
    b = full_run_digest.check_engine_run(eng, g, "c3lit")
    assert (b["status"] == 1).any(), "the literal mode binds OverCapacity pods"


def test_c3_full_trace_batch_independent_and_invariants(c3):
    tr, enc = c3
    m, n = tr["pods"]["m"], tr["nodes"]["n"]
    a = make_engine(tr, enc, MODE)             # default batch
    a.submit(enc["pods"])
    b = make_engine(tr, enc, MODE, batch_pods=97)
    b.submit(enc["pods"])
    dur = _dur_ticks(enc, tr["tick_seconds"])
    done, last_tick, allb = 0, 0, []
    for chunk in (200_000,) * 5:
        ea = a.step(chunk)
        eb = b.step(chunk)
        np.testing.assert_array_equal(ea, eb)
        _check_invariants(ea, done, n, enc, last_tick)
        allb.append(ea)
        done += len(ea)
        last_tick = int(ea["tick"][-1])
        sofar = np.concatenate(allb)
        _check_capacity(sofar, enc, dur, last_tick, n)
        _check_capacity(sofar, enc, dur, last_tick - 4321, n)
    assert done == m
    # the per-tick usage digest against ks_usage_at at sampled ticks of the last 100k ticks
    lo = last_tick - 100_000
    dg = a.usage_digest(lo, last_tick + 1)
    for t in (lo, lo + 1, lo + 31_337, last_tick - 1, last_tick):
        u = a.usage_at(t)
        np.testing.assert_array_equal(dg[t - lo, :3], u.sum(axis=0).astype(np.uint64))


def _group_step_all(g, ticks, chunk):
    out = None
    left = ticks
    while left > 0:
        k = min(chunk, left)
        binds, cnt, st, _ = g.step(k)
        parts = g.split(binds, cnt)
        out = parts if out is None else [np.concatenate([x, y]) for x, y in zip(out, parts)]
        left -= k
        if (st != 0).all():
            break
    return out, st


def test_c4_1024_scenarios_config_size():
    from kubesim_amd.engine import Group
    S, N, P = 1024, 2000, 10_000
    g = Group(S)
    traces, encs = [], []
    for s in range(S):
        tr = tracegen.c4_scenario(s, n_nodes=N, n_pods=P)
        enc = encoded(tr)
        e = g.add(tick_seconds=tr["tick_seconds"], filter_mode=1, filters=7, scorers=SCORERS)
        e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
        e.submit(enc["pods"])
        traces.append(tr)
        encs.append(enc)
    per, st = _group_step_all(g, P, 2500)
    with open(os.path.join(os.path.dirname(__file__), "golden", "c4_golden.json")) as f:
        gold = json.load(f)
    assert (gold["scenarios"], gold["nodes"], gold["pods"]) == (S, N, P)
    # the abort count the oracle predicts for the whole group (NotFound runs stop as Run would)
    assert sum(1 for x in st if x != 0) == gold["aborted"]
    for s, rc, nb, bd, ud in gold["rows"]:
        b = per[s]
        assert int(st[s]) == rc, (s, int(st[s]), rc)
        assert len(b) == nb, (s, len(b), nb)
        _check_invariants(b, 0, N, encs[s])
        assert full_run_digest.bind_digest(b) == bd, f"scenario {s}: binds differ from the oracle's"
        assert full_run_digest.digest(g.members[s].usage().astype(np.int64)) == ud, f"scenario {s}: usage"
    # two scenarios also directly against the oracle (the golden's own generator path)
    for s in (0, S - 1):
        ora = make_oracle(traces[s], MODE)
        ora.set_threads(_threads())
        ora.submit(traces[s])
        ob, rc = ora.step(P, cap=P)
        assert rc == int(st[s]), (s, rc, st[s])
        assert_same_binds(per[s], ob)
    g.close()
