"""GPU parity: the HIP engine (through the C-ABI) vs the CPU oracle, bit for bit.

Placements, bind order, bind ticks, bind status and per-tick node usage must be identical
(integer work: no tolerance).  Sizes are small enough for the oracle to finish in seconds;
full-size configs are covered by size-independent invariants in test_engine_gpu_large.py.
"""
import json
import os

import numpy as np
import pytest

from harness import (MODES, assert_same_binds, encoded, engine_run, make_engine, make_oracle,
                     oracle_run, small_trace)
from kubesim_amd import tracegen

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _lockstep(trace, mode, ticks, batch_pods=0, usage_every=1, chunk=1, engine_flags=0):
    enc = encoded(trace)
    eng = make_engine(trace, enc, mode, batch_pods, engine_flags)
    eng.submit(enc["pods"])
    ora = make_oracle(trace, mode)
    ora.submit(trace)
    t = 0
    while t < ticks:
        k = min(chunk, ticks - t)
        eb, erc = engine_run(eng, k, k)
        ob, orc = oracle_run(ora, k)
        assert_same_binds(eb, ob)
        assert erc == orc, (t, erc, orc, eng.tick, ora.tick)
        t += k
        if erc:
            break
        if usage_every and (t // chunk) % usage_every == 0:
            np.testing.assert_array_equal(eng.usage(), ora.usage(), err_msg=f"usage at tick {t}")
    return eng, ora


def test_c1_kat():
    """config/sample.yml + examples/main.go: even pods Ok on node-0, odd OverCapacity."""
    with open(os.path.join(GOLDEN, "c1_kat.json")) as f:
        kat = json.load(f)
    tr = tracegen.c1_trace(kat["ticks"])
    enc = encoded(tr)
    eng = make_engine(tr, enc, "literal_const")
    eng.submit(enc["pods"])
    for t, exp in enumerate(kat["binds"], start=1):
        b = eng.step(1)
        assert [(int(x["pod"]), int(x["node"]), int(x["tick"]), int(x["status"])) for x in b] == [tuple(exp)]
        np.testing.assert_array_equal(eng.usage(), np.array(kat["usage"][t - 1], dtype=np.int64))


@pytest.mark.parametrize("wide", [0, 1, 2, 4])
@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("seed", [1, 2])
def test_lockstep_small(mode, seed, wide):
    """Every evaluator variant against the oracle: 0 = engine's choice (micro 24-bit for these
    capacities), 1 = forced 64/128-bit, 2 = no tiny (narrow 32x32->64), 4 = no micro (tiny)."""
    tr = small_trace(seed, n_nodes=400, n_pods=300, arrival="stream")
    _lockstep(tr, mode, 400, engine_flags=wide)


def test_micro_lr_floor_selftest():
    """The micro evaluator's correction-free LeastRequested floor, every (x, A) pair with
    0 <= x <= A < 2^16, on the device (ks_selftest)."""
    from kubesim_amd.engine import selftest
    assert selftest() == 0


def test_micro_capacity_sweep_scores_match_oracle():
    """Every cpu capacity 1..65535 milli-units (the whole micro domain) with memory 1..255 MiB
    (Ac * Am up to the 2^24 edge): filter and score of pods with small and large requests match
    the oracle node for node."""
    n = 65535
    tr = small_trace(47, n_nodes=n, n_pods=24, taints=False, labels=False, tolerations=False, selectors=False)
    nd, p = tr["nodes"], tr["pods"]
    nd["alloc"][:, 0] = np.arange(1, n + 1)
    nd["alloc"][:, 1] = ((np.arange(n) * 7919) % 255 + 1) << 20
    nd["alloc"][:, 3] = 110
    nd["alloc_has"][:] |= 11  # cpu, memory, pods
    req_c = [0, 1, 2, 3, 5, 7, 10, 64, 99, 100, 255, 1000, 4095, 4096, 9999, 32767, 32768, 65534, 65535,
             70000, 1, 500, 12345, 60000]
    p["req"][:, 0] = req_c[: p["m"]]
    p["req"][:, 1] = (np.arange(p["m"]) * 37 % 256) << 20
    p["req_has"][:] |= 3
    mode = "feeds_all_lrba"
    enc = encoded(tr)
    eng = make_engine(tr, enc, mode)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    for pod in range(p["m"]):
        feas, score = ora.eval(pod)
        np.testing.assert_array_equal(eng.filter(pod), feas)
        np.testing.assert_array_equal(eng.score(pod), score, err_msg=f"pod {pod}")
    eb, erc = engine_run(eng, p["m"], p["m"])
    ob, orc = oracle_run(ora, p["m"])
    assert erc == orc
    assert_same_binds(eb, ob)


def test_narrow_capacities_use_narrow_evaluator():
    """cpu x memory beyond the tiny range (2^26 scaled units) but within the narrow one."""
    tr = small_trace(43, n_nodes=300, n_pods=600, taints=False, selectors=False, tolerations=False)
    nd = tr["nodes"]
    nd["alloc"][::2, 0] = 120_001 + 3 * np.arange(len(nd["alloc"][::2]))  # cpu unit 1m: ~2^17 x 2^11
    _lockstep(tr, "feeds_all_lrba", 600, batch_pods=128, chunk=150)


def test_wide_capacities_use_general_evaluator():
    """Capacities beyond the narrow range (2^29 units after scaling) must still be exact."""
    tr = small_trace(41, n_nodes=300, n_pods=600, taints=False, selectors=False, tolerations=False)
    nd = tr["nodes"]
    nd["alloc"][::3, 1] = (1 << 50) + 7 * np.arange(len(nd["alloc"][::3]))  # odd memory sizes, gcd 1
    _lockstep(tr, "feeds_all_lrba", 600, batch_pods=128, chunk=150)


def test_golden_small_traces_engine():
    """Committed fixtures (tests/golden/small_traces.json) — no oracle at run time."""
    from golden_traces import check_case
    with open(os.path.join(GOLDEN, "small_traces.json")) as f:
        gold = json.load(f)
    for case in gold["cases"]:
        check_case(case, "engine")


@pytest.mark.parametrize("batch", [1, 3, 64, 200, 256])
@pytest.mark.parametrize("mode", ["literal_lrba_filters_ignored", "feeds_all_lrba"])
def test_batched_vs_oracle(mode, batch):
    tr = small_trace(7, n_nodes=300, n_pods=2500, taints=False, selectors=False)
    enc = encoded(tr)
    eng = make_engine(tr, enc, mode, batch)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    for chunk in (1, 17, 500, 2000):
        eb, erc = engine_run(eng, chunk, chunk)
        ob, orc = oracle_run(ora, chunk)
        assert_same_binds(eb, ob)
        assert erc == orc
        np.testing.assert_array_equal(eng.usage(), ora.usage())


def test_short_pods_many_expiries():
    """Durations of 1-3 ticks: every pod expires inside its own batch; exercises the
    in-batch expiry path and the cache budget (early commits)."""
    tr = small_trace(11, n_nodes=2000, n_pods=6000, taints=False, selectors=False, tolerations=False)
    p = tr["pods"]
    p["phase_sec"][:] = 1 + (np.arange(len(p["phase_sec"])) % 12)
    _lockstep(tr, "feeds_all_lrba", 6000, batch_pods=256, chunk=1500)


def test_filter_score_match_oracle():
    tr = small_trace(5, n_nodes=64, n_pods=300)
    mode = "feeds_all_lrba"
    enc = encoded(tr)
    eng = make_engine(tr, enc, mode)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    for ticks in (0, 13, 40):
        engine_run(eng, ticks, ticks) if ticks else None
        oracle_run(ora, ticks) if ticks else None
        done = tr["pods"]["m"] - eng.queued
        for pod in (done, done + 1, done + 7):
            feas, score = ora.eval(pod)
            np.testing.assert_array_equal(eng.filter(pod), feas)
            np.testing.assert_array_equal(eng.score(pod), score)


def test_list_exhaustion_forces_rescan():
    """Identical nodes and pods under LeastRequested: pod k takes node k, so after L binds a
    pod's whole snapshot top-L list is touched and the batch must commit early and rescan."""
    tr = small_trace(21, n_nodes=300, n_pods=900, taints=False, labels=False, tolerations=False,
                     selectors=False)
    nd, p = tr["nodes"], tr["pods"]
    p["req"][:] = p["req"][0]
    nd["alloc"][:, :3] = 4 * p["req"][0]   # each bind drops the node's LeastRequested score
    nd["alloc"][:, 3] = 110
    nd["alloc_has"][:] = 15
    mode = "feeds_fit_lr"
    enc = encoded(tr)
    eng = make_engine(tr, enc, mode, 256)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    eb, erc = engine_run(eng, 900, 900)
    ob, orc = oracle_run(ora, 900)
    assert_same_binds(eb, ob)
    assert erc == orc
    assert eng.last_step_stats()["launches"] > 900 // 256 + 2  # early commits happened


def test_memory_unit_rescale_mid_run():
    """Memory is held in bytes while every quantity is whole bytes; a later pod requesting a
    fractional byte (e.g. memory "1.5") switches the device to milli-bytes mid-run.  Results
    must not change."""
    tr = small_trace(31, n_nodes=500, n_pods=1200, taints=False, selectors=False, tolerations=False)
    tr["pods"]["req"][700:, 1] += 1  # +1 milli-byte: not a whole byte
    mode = "feeds_all_lrba"
    enc = encoded(tr)
    eng = make_engine(tr, enc, mode, 256)
    ora = make_oracle(tr, mode)
    from kubesim_amd import encode as E
    for lo, hi in ((0, 600), (600, 1200)):
        part = tracegen.slice_pods(tr, lo, hi)
        eng.submit(E.encode_pods(part["pods"], enc["taint_dict"], enc["label_dict"]))
        ora.submit(part)
        eb, erc = engine_run(eng, 600, 600)
        ob, orc = oracle_run(ora, 600)
        assert_same_binds(eb, ob)
        assert erc == orc
        np.testing.assert_array_equal(eng.usage(), ora.usage())


# ---- node sharding: per-shard top-L lists merged after an exchange ----------
@pytest.mark.parametrize("vshards", [2, 3, 8])
def test_virtual_shards_match_oracle(vshards):
    """One rank, several node shards: the per-shard scan + merge + shard merge path."""
    tr = small_trace(21, n_nodes=1500, n_pods=3000, taints=True, selectors=True)
    enc = encoded(tr)
    mode = "feeds_all_lrba"
    eng = make_engine(tr, enc, mode, 256, shard=(1, 0, None, vshards))
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    for chunk in (700, 2300):
        eb, erc = engine_run(eng, chunk, chunk)
        ob, orc = oracle_run(ora, chunk)
        assert_same_binds(eb, ob)
        assert erc == orc
        np.testing.assert_array_equal(eng.usage(), ora.usage())


def test_rccl_exchange_single_rank():
    """The RCCL all-gather path with a one-rank communicator (two virtual shards)."""
    from kubesim_amd.engine import comm_unique_id
    tr = small_trace(22, n_nodes=700, n_pods=1500)
    enc = encoded(tr)
    mode = "literal_lrba_filters_ignored"
    eng = make_engine(tr, enc, mode, 128, shard=(1, 0, comm_unique_id(), 2))
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    eb, erc = engine_run(eng, 1500, 1500)
    ob, orc = oracle_run(ora, 1500)
    assert_same_binds(eb, ob)
    assert erc == orc


def test_shard_geometry_rejected():
    from kubesim_amd.engine import Engine, KsError
    eng = Engine()
    with pytest.raises(KsError):
        eng.shard(2, 0, None)  # world > 1 needs a communicator
    with pytest.raises(KsError):
        eng.shard(1, 1, None)
    eng.load_nodes(np.array([[1000, 1000, -1, 10]]), np.zeros(1, np.uint64), np.zeros(1, np.uint64))
    with pytest.raises(KsError):
        eng.shard(1, 0, None, 2)  # after load_nodes


# ---- scenario groups (BASELINE.json configs[3]): what-if clusters side by side in one launch ----
def test_group_scenarios_match_oracle():
    """Scenarios of different sizes, traces and outcomes (one aborts with NotFound) stepped
    together; each must equal its own oracle run, and an aborted member must not disturb the
    others."""
    from kubesim_amd.engine import Group
    mode = "feeds_all_lrba"
    fm, fl, sc = MODES[mode]
    specs = [(0, 300, 900), (1, 700, 1200), (2, 64, 800), (3, 1500, 600), (4, 200, 1000)]
    g = Group(len(specs))
    runs = []
    for s, n, p in specs:
        tr = tracegen.c4_scenario(s, n_nodes=n, n_pods=p)
        enc = encoded(tr)
        e = g.add(tick_seconds=tr["tick_seconds"], filter_mode=fm, filters=fl, scorers=sc, batch_pods=256)
        e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
        e.submit(enc["pods"])
        o = make_oracle(tr, mode)
        o.submit(tr)
        runs.append((e, o))
    aborted = 0
    for chunk in (250, 1000):
        allb, cnt, st, stats = g.step(chunk)
        for (e, o), eb, rc in zip(runs, g.split(allb, cnt), st):
            ob, orc = oracle_run(o, chunk)
            assert_same_binds(eb, ob)
            assert rc == orc
            aborted += rc != 0
            if rc == 0:
                np.testing.assert_array_equal(e.usage(), o.usage())
    assert stats["launches"] >= 1
    g.close()


def test_group_member_steps_alone_too():
    """A member can still be stepped on its own (ks_step) and agrees with the group path."""
    from kubesim_amd.engine import Group
    mode = "feeds_all_lrba"
    fm, fl, sc = MODES[mode]
    tr = tracegen.c4_scenario(9, n_nodes=500, n_pods=700)
    enc = encoded(tr)
    g = Group(2)
    a = g.add(tick_seconds=10, filter_mode=fm, filters=fl, scorers=sc)
    b = g.add(tick_seconds=10, filter_mode=fm, filters=fl, scorers=sc)
    for e in (a, b):
        e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
        e.submit(enc["pods"])
    a1, rc1 = engine_run(a, 300, 300)  # member alone: ticks 1..300
    o = make_oracle(tr, mode)
    o.submit(tr)
    ob1, orc1 = oracle_run(o, 300)
    assert_same_binds(a1, ob1)
    assert rc1 == orc1 == 0
    allb, cnt, st, _ = g.step(300)     # a: ticks 301..600, b: ticks 1..300
    a2, b1 = g.split(allb, cnt)
    np.testing.assert_array_equal(a1, b1)
    assert st[1] == 0
    ob2, orc2 = oracle_run(o, 300)     # the oracle may stop with NotFound: so must `a`
    assert_same_binds(a2, ob2)
    assert st[0] == orc2
    g.close()


# ---- pod status: Pod.BuildStatus phases -----------------------------------
def test_pod_status_matches_reference_rules():
    """Phases from the oracle's binds restated with the reference's rules (kubesim/pod/pod.go:
    67-69 IsRunning, 78-145 BuildStatus): FAILED for OverCapacity, RUNNING while
    (t - t0) * tick < Σ phase seconds, else SUCCEEDED; PENDING when not bound."""
    from kubesim_amd import _lib
    tr = small_trace(13, n_nodes=60, n_pods=900, arrival="stream")
    mode = "literal_lrba_filters_ignored"  # filters ignored: OverCapacity binds happen
    enc = encoded(tr)
    eng = make_engine(tr, enc, mode)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    p = tr["pods"]
    S = np.add.reduceat(p["phase_sec"].astype(np.int64), p["phase_off"][:-1]) if len(p["phase_sec"]) else None
    S = np.where(np.diff(p["phase_off"]) > 0, S, 0).astype(np.int64)
    S32 = ((S + 2**31) % 2**32 - 2**31).astype(np.int64)  # int32 wrapping sum (pod.go:155-162)
    binds = []
    for ticks in (150, 400, 1200):
        eb, erc = engine_run(eng, ticks, ticks)
        ob, orc = oracle_run(ora, ticks)
        assert_same_binds(eb, ob)
        binds.append(eb)
        allb = np.concatenate(binds)
        st = eng.pod_status()
        t = eng.tick
        exp = np.full(p["m"], _lib.KS_PHASE_PENDING)
        q = allb["pod"]
        ok = allb["status"] == 0
        running = ok & ((t - allb["tick"]) * tr["tick_seconds"] < S32[q])
        exp[q] = np.where(~ok, _lib.KS_PHASE_FAILED, np.where(running, _lib.KS_PHASE_RUNNING, _lib.KS_PHASE_SUCCEEDED))
        np.testing.assert_array_equal(st["phase"], exp)
        np.testing.assert_array_equal(st["node"][q], allb["node"])
        np.testing.assert_array_equal(st["start_tick"][q], allb["tick"])
        np.testing.assert_array_equal(st["total_seconds"], S32)
        assert (st["phase"] == _lib.KS_PHASE_FAILED).any() or ticks < 1200
        if erc:
            break


# ---- host ingest end to end: YAML / Quantity / simSpec text -> engine ----
def test_c1_from_text_through_ingest():
    """config/sample.yml's cluster and examples/main.go's pods given as TEXT, parsed by the C++
    ingest (ks_cluster_parse, ks_parse_quantity, ks_parse_simspec) and scheduled on the device:
    the committed C1 KAT (tests/golden/c1_kat.json) must come out."""
    from kubesim_amd.engine import Engine
    from kubesim_amd.ingest import Cluster, parse_quantity, parse_simspec
    from test_ingest import CONFIG, K
    with open(os.path.join(GOLDEN, "c1_kat.json")) as f:
        kat = json.load(f)
    cfg = CONFIG[:CONFIG.index("  - namespace: other")]            # node-0, node-1 of the sample
    cfg = cfg[:cfg.index("    taints:")]                          # without the extra taints
    c = Cluster(cfg)
    eng = Engine(tick_seconds=c.tick, filter_mode=0, filters=0, scorers=((0, 1, 1),))
    eng.load_nodes(c.alloc, c.taint, c.label)
    inp = K["c1_inputs"]
    req = [parse_quantity(inp["pod_requests"][k])[1] for k in ("cpu", "memory", "nvidia.com/gpu")]
    phases = parse_simspec(inp["sim_spec"])
    m = kat["ticks"]
    names = ("cpu", "memory", "nvidia.com/gpu")
    pods = dict(m=m, arrival=np.arange(1, m + 1), req=np.tile(req, (m, 1)), keymask=np.full(m, 7, np.uint8),
                tol=np.zeros(m, np.uint64), sel=np.zeros(m, np.uint64),
                phase_off=np.arange(0, len(phases) * m + 1, len(phases), dtype=np.int32),
                phase_sec=np.tile([s for s, _ in phases], m).astype(np.int32),
                phase_use=np.tile([[u.get(k, 0) for k in names] for _, u in phases], (m, 1)),
                flags=np.zeros(m, np.uint8))
    eng.submit(pods)
    for t, exp in enumerate(kat["binds"], start=1):
        b = eng.step(1)
        assert [(int(x["pod"]), int(x["node"]), int(x["tick"]), int(x["status"])) for x in b] == [tuple(exp)]
        np.testing.assert_array_equal(eng.usage(), np.array(kat["usage"][t - 1], dtype=np.int64))
