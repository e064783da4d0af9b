"""The engine's int32 passed-seconds domain ("what's missing" 5).

Pod.passedSeconds = int32(clock.Sub(start).Seconds()) (kubesim/pod/pod.go:148-153); past 2^31 s
Go's float -> int32 conversion is implementation-defined and IsRunning (pod.go:67-69) may revive
a finished pod.  The engine refuses, with KS_ERANGE and nothing changed, any step or submit that
would evaluate a tick 2^31 s or more after the run's first bind; the oracle refuses the same tick
(tests/test_oracle.py::test_oracle_refuses_ticks_past_int32_passed_seconds).  A tick of 2^20 s
puts the boundary 2047 ticks after the first bind.
"""
import numpy as np
import pytest

from harness import assert_same_binds, encoded, make_engine, make_oracle, small_trace

pytestmark = pytest.mark.gpu
MODE = "feeds_all_lrba"
TICK = 1 << 20
SPAN = (2**31 - 1) // TICK   # ticks after the first bind still inside the domain


def _trace():
    tr = small_trace(5, n_nodes=32, n_pods=40, arrival="stream", selectors=False)
    tr["tick_seconds"] = TICK
    return tr


def test_step_past_domain_refused_then_queries_still_work():
    from kubesim_amd import _lib
    from kubesim_amd.engine import KsError
    tr = _trace()
    enc = encoded(tr)
    eng = make_engine(tr, enc, MODE)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, MODE)
    ora.submit(tr)
    eb = eng.step(200)
    ob, rc = ora.step(200)
    assert rc == 0
    assert_same_binds(eb, ob)
    t0 = int(eb["tick"][0])
    last = t0 + SPAN
    eng.step(last - eng.tick)
    ora.step(last - ora.tick)
    assert eng.tick == last
    np.testing.assert_array_equal(eng.usage(), ora.usage())
    with pytest.raises(KsError) as ex:
        eng.step(1)
    assert ex.value.code == _lib.KS_ERANGE
    assert eng.tick == last
    _, rc = ora.step(1)
    assert rc == _lib.KS_ERANGE
    # not sticky: queries and zero-tick steps still answer
    np.testing.assert_array_equal(eng.usage(), ora.usage())
    assert len(eng.step(0)) == 0


def test_submit_past_domain_refused_atomically():
    from kubesim_amd import _lib, tracegen
    from kubesim_amd.engine import KsError
    tr = _trace()
    enc = encoded(tr)
    eng = make_engine(tr, enc, MODE)
    eng.submit(enc["pods"])
    first = int(eng.step(1)["tick"][0])
    m0 = eng.queued
    late = dict(encoded(tracegen.slice_pods(tr, 0, 3))["pods"])
    if late.get("key_id") is not None:
        late["key_id"] = np.arange(3, dtype=np.int64) + 10**6   # fresh keys: only the domain matters
    late["arrival"] = np.array([first + SPAN - 1, first + SPAN, first + SPAN + 1], np.int64)
    with pytest.raises(KsError) as ex:
        eng.submit(late)
    assert ex.value.code == _lib.KS_ERANGE
    assert eng.queued == m0                    # nothing appended
    late["arrival"] = np.array([first + SPAN - 2, first + SPAN - 1, first + SPAN], np.int64)
    eng.submit(late)                           # the last bind tick is exactly the domain's end
    assert eng.queued == m0 + 3


def test_multi_tick_step_crossing_the_domain_refused_whole_on_both():
    """one ks_step(N) / ko_step(N) whose end leaves the domain — both refuse it before
    any tick runs (same binds, same tick, same usage after)."""
    from kubesim_amd import _lib
    from kubesim_amd.engine import KsError
    tr = _trace()
    enc = encoded(tr)
    eng = make_engine(tr, enc, MODE)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, MODE)
    ora.submit(tr)
    eb = eng.step(30)
    ob, rc = ora.step(30)
    assert rc == 0
    assert_same_binds(eb, ob)
    last = int(eb["tick"][0]) + SPAN
    with pytest.raises(KsError) as ex:
        eng.step(last - eng.tick + 3)
    assert ex.value.code == _lib.KS_ERANGE
    b, rc = ora.step(last - ora.tick + 3)
    assert rc == _lib.KS_ERANGE and len(b["pod"]) == 0
    assert eng.tick == ora.tick
    np.testing.assert_array_equal(eng.usage(), ora.usage())
    eb = eng.step(last - eng.tick)
    ob, rc = ora.step(last - ora.tick)
    assert rc == 0
    assert_same_binds(eb, ob)
