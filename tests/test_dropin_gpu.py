"""The drop-in's own call sequence on the device.

go/kubesim/engine/kubesim.go's Run issues, per tick, the submitters' pods to ks_submit_pods with
arrival = the tick and then ks_step(1) (kubesim/kubesim.go:90-123 restated); RunWindowed calls
placement-blind submitters `window` ticks ahead and steps once.  kubesim_amd.kubesim.KubeSim is
that loop call for call (no Go toolchain here or on the box), and this file checks both forms
bind-for-bind against the reference's KAT and the oracle, with ks_filter / ks_score probed on
the queue head every tick as the api.Filter / api.Scorer adapters would.  The rates are printed
(bench.py reports them in its line under "dropin").
"""
import json
import os
import time

import numpy as np
import pytest

from harness import assert_same_binds, encoded, make_engine, make_oracle, small_trace
from kubesim_amd import tracegen
from kubesim_amd.kubesim import KubeSim, TraceSubmitter, head_probe

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _sim(tr, enc, mode, **kw):
    eng = make_engine(tr, enc, mode, **kw)
    ks = KubeSim(eng, tr["tick_seconds"])
    ks.register_submitter(TraceSubmitter(enc["pods"]))
    return ks


@pytest.mark.parametrize("windowed", [False, True])
def test_c1_kat_through_the_run_loop(windowed):
    with open(os.path.join(GOLDEN, "c1_kat.json")) as f:
        kat = json.load(f)
    T = kat["ticks"]
    tr = tracegen.c1_trace(T)
    enc = encoded(tr)
    ks = _sim(tr, enc, "literal_const")
    if windowed:
        ks.run_windowed(T, 16)
    else:
        ks.run(T, probe=head_probe)
    b = ks.all_binds()
    got = [[int(x["pod"]), int(x["node"]), int(x["tick"]), int(x["status"])] for x in b]
    assert got == kat["binds"]
    np.testing.assert_array_equal(ks.eng.usage(), np.array(kat["usage"][T - 1]))
    if not windowed:
        assert ks.calls["step"] == T and ks.calls["probe"] == T


def test_c2_prefix_per_tick_and_windowed_equal_oracle():
    """5k nodes, stream arrivals (0-2 ticks apart): per-tick Run, windowed Run and the oracle."""
    P, T = 1500, 1600
    tr = tracegen.c2_trace(n_pods=P, arrival="stream")
    enc = encoded(tr)
    mode = "feeds_all_lrba"
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    ob, rc = ora.step(T, cap=T)
    assert rc == 0

    ks = _sim(tr, enc, mode)
    t0 = time.perf_counter()
    ks.run(T)
    dt_tick = time.perf_counter() - t0
    assert_same_binds(ks.all_binds(), ob)
    np.testing.assert_array_equal(ks.eng.usage(), ora.usage())

    ks2 = _sim(tr, enc, mode)
    t0 = time.perf_counter()
    ks2.run_windowed(T, 256)
    dt_win = time.perf_counter() - t0
    assert_same_binds(ks2.all_binds(), ob)
    np.testing.assert_array_equal(ks2.eng.usage(), ora.usage())

    ks3 = _sim(tr, enc, mode)
    t0 = time.perf_counter()
    ks3.run(300, probe=head_probe)
    dt_probe = time.perf_counter() - t0
    assert_same_binds(ks3.all_binds(), {k: v[:len(ks3.all_binds())] for k, v in ob.items()})
    n = len(ob["pod"])
    print(f"\ndrop-in C2 prefix: per-tick Run {n / dt_tick:.0f} pods/s ({dt_tick / T * 1e6:.0f} us/tick), "
          f"windowed(256) {n / dt_win:.0f} pods/s, per-tick + filter/score probe "
          f"{dt_probe / 300 * 1e6:.0f} us/tick")


def test_windowed_refuses_placement_aware_submitters():
    tr = tracegen.c1_trace(10)
    enc = encoded(tr)
    ks = _sim(tr, enc, "literal_const")
    ks.register_submitter(lambda t, c: None)   # no placement_blind declaration
    with pytest.raises(ValueError):
        ks.run_windowed(10, 4)


# ---- the C++ Run loop (include/ks_kubesim.h) and the per-tick path (ks_tick.hip) --------------
def _native(tr, enc, mode, **kw):
    from kubesim_amd.kubesim import NativeRun
    eng = make_engine(tr, enc, mode, **kw)
    return NativeRun(eng, enc["pods"], tr["tick_seconds"])


@pytest.mark.parametrize("window", [1, 16])
def test_c1_kat_through_the_native_run_loop(window):
    with open(os.path.join(GOLDEN, "c1_kat.json")) as f:
        kat = json.load(f)
    T = kat["ticks"]
    tr = tracegen.c1_trace(T)
    nr = _native(tr, encoded(tr), "literal_const")
    b, _ = nr.run(T, window)
    got = [[int(x["pod"]), int(x["node"]), int(x["tick"]), int(x["status"])] for x in b]
    assert got == kat["binds"]
    np.testing.assert_array_equal(nr.eng.usage(), np.array(kat["usage"][T - 1]))


@pytest.mark.parametrize("window", [1, 64])
def test_c2_prefix_native_run_equals_oracle(window):
    P, T = 2000, 2100
    tr = tracegen.c2_trace(n_pods=P, arrival="stream")
    enc = encoded(tr)
    mode = "feeds_all_lrba"
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    ob, rc = ora.step(T, cap=T)
    assert rc == 0
    nr = _native(tr, enc, mode)
    b, sec = nr.run(T, window)
    assert_same_binds(b, ob)
    np.testing.assert_array_equal(nr.eng.usage(), ora.usage())
    print(f"\nnative Run window {window}: {len(b) / sec:.0f} pods/s ({sec / T * 1e6:.1f} us/tick)")


@pytest.mark.parametrize("window", [1, 16])
def test_native_run_submit_error_steps_the_ticks_before_it(window):
    """a submit that fails at tick t (a request outside the exact domain: KS_EINVAL from
    ks_submit_pods) stops Run after it has scheduled every tick before t — also with window > 1,
    where the ticks since the last step are stepped before the error returns."""
    from kubesim_amd import _lib
    from kubesim_amd.engine import KsError
    P, T = 300, 400
    tr = tracegen.c2_trace(n_pods=P, arrival="stream")
    enc = encoded(tr)
    bad = 137
    enc["pods"]["req"] = np.array(enc["pods"]["req"], copy=True)
    enc["pods"]["req"].reshape(-1, 3)[bad, 0] = 1 << 60
    t_bad = int(enc["pods"]["arrival"][bad])
    mode = "feeds_all_lrba"
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    ob, rc = ora.step(t_bad - 1, cap=T)  # Run's binds before tick t_bad
    assert rc == 0
    nr = _native(tr, enc, mode)
    with pytest.raises(KsError) as ex:
        nr.run(T, window)
    assert ex.value.code == _lib.KS_EINVAL
    assert_same_binds(ex.value.binds, ob)
    assert nr.eng.tick == t_bad - 1
    np.testing.assert_array_equal(nr.eng.usage(), ora.usage())


def test_tick_path_dense_expiries_mixed_steps_and_probes():
    """Short phases (many expiries due per tick), one pod per tick: ks_step(1) takes the one-launch
    path, its by-value expiry list and the host-staged submits; interleaved with batched steps
    (the batch path must see the same device state) and filter/score probes (the exact host flush
    list) — every bind, the usage and the probes against the oracle."""
    tr = small_trace(11, n_nodes=600, n_pods=3000, taints=False, selectors=False, tolerations=False)
    p = tr["pods"]
    p["phase_sec"][:] = 1 + (np.arange(len(p["phase_sec"])) % 40)
    p["arrival"][:] = np.arange(1, p["m"] + 1)
    enc = encoded(tr)
    mode = "feeds_all_lrba"
    eng = make_engine(tr, enc, mode)
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    ks = KubeSim(eng, tr["tick_seconds"])
    ks.register_submitter(TraceSubmitter(enc["pods"]))
    t = 0
    for phase, (k, per_tick) in enumerate([(400, True), (700, False), (300, True), (900, False), (200, True)]):
        if per_tick:
            ks.run(k)
        else:
            ks.run_windowed(k, k)
        ob, rc = ora.step(k, cap=k)
        assert rc == 0
        got = ks.all_binds()[-len(ob["pod"]):] if len(ob["pod"]) else ks.all_binds()[:0]
        assert_same_binds(got, ob)
        np.testing.assert_array_equal(eng.usage(), ora.usage(), err_msg=f"phase {phase}")
        t += k
        q = min(eng._submitted - eng.queued, eng._submitted - 1)  # the queue head, else the last pod
        if q >= 0:
            feas, score = ora.eval(q)
            np.testing.assert_array_equal(eng.filter(q), feas)
            np.testing.assert_array_equal(eng.score(q), score)


@pytest.mark.parametrize("mode,code", [("no_scorers", 2), ("bad_spec", 1)])
def test_tick_path_stops_as_run(mode, code):
    """NotFound (no candidate) and a bad simSpec stop Run at that pod's tick (kubesim.go:217-220,
    pod.go:31-39): the per-tick path returns the same error, binds and tick as the oracle."""
    from kubesim_amd.engine import KsError
    tr = small_trace(5, n_nodes=64, n_pods=40, selectors=False)  # (a selector no node carries: NotFound)
    tr["pods"]["arrival"][:] = np.arange(1, 41)
    m = "feeds_all_lrba"
    if mode == "bad_spec":
        tr["pods"]["flags"][17] = 2
    else:
        m = "no_scorers"
    enc = encoded(tr)
    ora = make_oracle(tr, m)
    ora.submit(tr)
    ob, orc = ora.step(60, cap=60)
    eng = make_engine(tr, enc, m)
    ks = KubeSim(eng, tr["tick_seconds"])
    ks.register_submitter(TraceSubmitter(enc["pods"]))
    with pytest.raises(KsError) as ex:
        ks.run(60)
    assert ex.value.code == orc == code
    assert_same_binds(ks.all_binds(), ob)
    assert eng.tick == ora.tick
