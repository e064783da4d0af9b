"""GPU parity of the per-tick usage queries and of pod keys.

* ks_usage_at: usage at EVERY tick of one batched ks_step, against the oracle stepped tick by
  tick (Pod.ResourceUsage, kubesim/pod/pod.go:47-63, summed per node after each tick's bind);
* ks_usage_digest: the per-tick fingerprint of the same window, recomputed from the oracle's
  per-tick matrices (tests/usage_digest.py);
* pod keys: a key reused while its earlier pod may still run is refused (KS_ERANGE, nothing
  appended); reused keys of finished pods schedule exactly as the oracle, which models
  node.pods.Store's replacement (kubesim/node/node.go:58); Node.GetPod / GetPodList answers
  (ks_pod_lookup / ks_node_pods) follow the last Store per node and key.
"""
import numpy as np
import pytest

from harness import assert_same_binds, encoded, make_engine, make_oracle, oracle_run, small_trace
from usage_digest import digest_from_matrices

pytestmark = pytest.mark.gpu
MODE = "feeds_all_lrba"


def _short_trace(seed, n_nodes, n_pods, irregular=False):
    # no nodeSelectors: a pair no node of a small cluster carries stops the run with NotFound
    tr = small_trace(seed, n_nodes=n_nodes, n_pods=n_pods, arrival="stream", selectors=False)
    p = tr["pods"]
    F = len(p["phase_sec"])
    p["phase_sec"][:] = 1 + (np.arange(F) * 7919) % 97   # 1..97 s: phases change every few ticks
    if irregular:
        # a negative phase and one that wraps the int32 sum: the digest's per-tick path and the
        # reference's int32 arithmetic
        off = p["phase_off"]
        multi = np.nonzero(np.diff(off) >= 2)[0]
        p["phase_sec"][off[multi[3]]] = -25
        p["phase_sec"][off[multi[7]]] = 2**31 - 40
        p["phase_sec"][off[multi[7]] + 1] = 100
    return tr


@pytest.mark.parametrize("irregular", [False, True])
def test_usage_at_every_tick_of_one_batched_step(irregular):
    T = 2000
    tr = _short_trace(31, 96, 2400, irregular)
    enc = encoded(tr)
    eng = make_engine(tr, enc, MODE, batch_pods=128)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, MODE)
    ora.submit(tr)
    per_tick, obinds = [], []
    for _ in range(T):
        b, rc = ora.step(1, cap=1)
        assert rc == 0
        obinds.append(b)
        per_tick.append(ora.usage())
    eb = eng.step(T)   # one batched step: ~2000 binds across many scan/resolve launches
    ob = {k: np.concatenate([x[k] for x in obinds]) for k in obinds[0]}
    assert_same_binds(eb, ob)
    assert eng.last_step_stats()["launches"] > 10
    np.testing.assert_array_equal(eng.usage_at(0), np.zeros((96, 3), np.int64))
    for t in range(1, T + 1):
        np.testing.assert_array_equal(eng.usage_at(t), per_tick[t - 1], err_msg=f"usage at tick {t}")
    np.testing.assert_array_equal(eng.usage(), per_tick[-1])
    want = digest_from_matrices(np.stack(per_tick))
    got = eng.usage_digest(1, T + 1)
    np.testing.assert_array_equal(got, want)
    # sub-windows and a window ending at the current tick
    np.testing.assert_array_equal(eng.usage_digest(700, 1300), want[699:1299])
    np.testing.assert_array_equal(eng.usage_digest(T, T + 1), want[-1:])


def test_usage_queries_reject_future_ticks():
    from kubesim_amd.engine import KsError
    tr = _short_trace(5, 32, 100)
    enc = encoded(tr)
    eng = make_engine(tr, enc, MODE)
    eng.submit(enc["pods"])
    eng.step(50)
    with pytest.raises(KsError):
        eng.usage_at(51)
    with pytest.raises(KsError):
        eng.usage_digest(10, 52)
    with pytest.raises(KsError):
        eng.usage_digest(10, 10)
    eng.usage_digest(1, 51)


def _bind_ticks(arrival, start_tick=0):
    bt, prev = [], start_tick
    for a in arrival:
        prev = max(prev + 1, int(a), start_tick + 1)
        bt.append(prev)
    return np.array(bt)


def _run_end(trace, tick_seconds=10):
    p = trace["pods"]
    off, sec = p["phase_off"], p["phase_sec"].astype(np.int64)
    S = np.array([sec[off[i]:off[i + 1]].sum() for i in range(p["m"])])
    return np.where(S > 0, -(-S // tick_seconds), 0)


def _reused_key_trace(seed, n_nodes=24, n_pods=600):
    """Keys reused as soon as the earlier pod with the key has surely finished."""
    tr = small_trace(seed, n_nodes=n_nodes, n_pods=n_pods, arrival="stream", selectors=False)
    p = tr["pods"]
    p["phase_sec"][:] = 1 + (np.arange(len(p["phase_sec"])) * 31) % 60
    bt = _bind_ticks(p["arrival"])
    end = bt + _run_end(tr)
    keys = np.zeros(p["m"], np.int64)
    key_end, nxt, reused = {}, 0, 0
    for j in range(p["m"]):
        cand = keys[j - 7] if j >= 7 else None
        if cand is not None and key_end[int(cand)] <= bt[j]:
            keys[j] = cand
            reused += 1
        else:
            keys[j] = 10_000 + nxt
            nxt += 1
        key_end[int(keys[j])] = max(key_end.get(int(keys[j]), 0), int(end[j]))
    p["key_id"] = keys
    assert reused > p["m"] // 6, reused
    return tr


def test_reused_keys_of_finished_pods_match_oracle():
    tr = _reused_key_trace(41)
    m = tr["pods"]["m"]
    enc = encoded(tr)
    eng = make_engine(tr, enc, MODE, batch_pods=64)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, MODE)
    ora.submit(tr)
    T = int(_bind_ticks(tr["pods"]["arrival"])[-1])
    eb = eng.step(T)
    ob, rc = oracle_run(ora, T)
    assert rc == 0
    assert_same_binds(eb, ob)
    np.testing.assert_array_equal(eng.usage(), ora.usage())
    # Node.GetPod / GetPodList: the last Store per (node, key)
    keys = tr["pods"]["key_id"]
    from kubesim_amd.engine import KsError
    for nd in range(tr["nodes"]["n"]):
        on = eb["pod"][eb["node"] == nd]
        last = {}
        for q in on:
            last[int(keys[q])] = int(q)
        np.testing.assert_array_equal(eng.node_pods(nd), np.array(sorted(last.values()), np.int64))
        for k, q in list(last.items())[:5]:
            assert eng.pod_lookup(nd, k) == q
    with pytest.raises(KsError) as ex:
        eng.pod_lookup(0, 123456789)
    assert ex.value.kind == "NotFound"
    assert m == len(eb)


def test_key_reused_while_running_is_refused():
    from kubesim_amd import _lib
    from kubesim_amd.engine import KsError
    tr = _reused_key_trace(43, n_pods=200)
    p = tr["pods"]
    enc = encoded(tr)
    eng = make_engine(tr, enc, MODE)
    # pod 150 takes the key of pod 149, which runs 50+ ticks from its bind (pod 150 binds at
    # most 3 ticks later)
    bad = dict(enc["pods"])
    bad["key_id"] = p["key_id"].copy()
    bad["key_id"][150] = bad["key_id"][149]
    bad["phase_sec"] = bad["phase_sec"].copy()
    off = bad["phase_off"]
    bad["phase_sec"][off[149]:off[150]] = 500
    with pytest.raises(KsError) as ex:
        eng.submit(bad)
    assert ex.value.code == _lib.KS_ERANGE
    assert eng.queued == 0          # nothing appended
    eng.submit(enc["pods"])        # the valid trace is still accepted afterwards
    assert eng.queued == p["m"]
    # across two submit calls: a later call reusing a running pod's key is refused too
    from kubesim_amd import tracegen
    more = encoded(tracegen.slice_pods(tr, 0, 10))["pods"]
    more["arrival"] = np.full(10, int(p["arrival"][-1]), np.int64)
    more["phase_sec"] = np.full_like(more["phase_sec"], 500)
    ok = dict(more, key_id=np.arange(10, dtype=np.int64) + 77_000)   # fresh distinct keys: fine
    more["key_id"] = np.full(10, 88_000, np.int64)                    # pod 1 reuses pod 0's key
    with pytest.raises(KsError) as ex:
        eng.submit(more)
    assert ex.value.code == _lib.KS_ERANGE
    assert eng.queued == p["m"]
    eng.submit(ok)
    assert eng.queued == p["m"] + 10
    more["key_id"] = np.full(10, 77_000, np.int64)                    # pod 0 reuses a running key
    with pytest.raises(KsError) as ex:
        eng.submit(more)
    assert ex.value.code == _lib.KS_ERANGE
    assert eng.queued == p["m"] + 10


def test_submit_checks_array_lengths():
    tr = _short_trace(7, 16, 50)
    enc = encoded(tr)
    eng = make_engine(tr, enc, MODE)
    bad = dict(enc["pods"])
    bad["tol"] = bad["tol"][:-1]
    with pytest.raises(ValueError):
        eng.submit(bad)
    bad = dict(enc["pods"])
    bad["phase_off"] = bad["phase_off"][:-1]
    with pytest.raises(ValueError):
        eng.submit(bad)
    eng.submit(enc["pods"])
    b = eng.step(10**8)            # cap defaults to the queued pods, not 10^8 rows (10^8 ticks of 10 s: inside the int32 passed-seconds domain)
    assert len(b) == 50
