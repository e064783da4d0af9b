"""GPU parity at BASELINE.json configs[4] size: the 1M-node cluster, node-sharded.

The 8-GPU layout (8 ranks x 131,072 nodes, candidate lists all-gathered over RCCL) cannot run on
one box, so its data path is exercised here with virtual shards: one engine splits the node range
into 8 parts, scans and merges each part to an exact per-pod top-L list, then runs the same second
merge the all-gather feeds (ks_engine.cpp, ks_shard).  Checked:
  * an exact prefix bind-for-bind and usage-for-usage against the CPU oracle
    (kubesim/kubesim.go:90-225) at 1M nodes: 2,000 pods (the OpenMP oracle needs a few ms per pod
    here on the box's 16 threads);
  * the WHOLE 196,608-pod trace (every pod the bench's C5 leg binds), sharded and unsharded,
    window by window against the oracle's committed digests (tests/golden/full_run.json);
  * the invariants of test_engine_gpu_large.py on the full run: FIFO one bind per tick, every
    bind Ok and satisfying the taint / selector filters, usage within capacity.
At 1M nodes the resolver's touched-node filter is the hashed one (nodes > the exact-bitmap range),
so this is also the full-size parity test of that path.
"""
import os

import numpy as np
import pytest

import full_run_digest
from harness import assert_same_binds, encoded, make_engine, make_oracle, oracle_run
from kubesim_amd import tracegen

pytestmark = pytest.mark.gpu
MODE = "feeds_all_lrba"
N_PODS = 196_608   # the pods bench.py's C5 leg binds (warm-up + 4 timed + 1 profiled steps)


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS") or 0) or min(os.cpu_count() or 1, 16)


@pytest.fixture(scope="module")
def c5():
    tr = tracegen.c5_trace(n_pods=N_PODS)
    return tr, encoded(tr)


def test_c5_sharded_prefix_matches_oracle(c5):
    tr, enc = c5
    eng = make_engine(tr, enc, MODE, shard=(1, 0, None, 8))
    eng.submit(enc["pods"])
    n = 2000
    ora = make_oracle(tr, MODE)
    ora.set_threads(_threads())
    ora.submit(tracegen.slice_pods(tr, 0, n))
    eb = eng.step(n)
    ob, orc = oracle_run(ora, n)
    assert orc == 0
    assert_same_binds(eb, ob)
    np.testing.assert_array_equal(eng.usage(), ora.usage())


def test_c5_whole_trace_sharded_and_unsharded_match_oracle_golden(c5):
    """Every pod the bench's C5 leg binds (196,608), window by window against the oracle's
    committed digests (tests/golden/full_run.json), both unsharded and with 8 virtual shards;
    plus the invariants on the full run."""
    tr, enc = c5
    g = full_run_digest.load("c5")
    if g is None:
        pytest.skip("tests/golden/full_run.json has no c5 run yet (tests/golden/make_full_run.py --only c5)")
    assert g["pods"] == tr["pods"]["m"] and g["nodes"] == tr["nodes"]["n"]
    a = make_engine(tr, enc, MODE, shard=(1, 0, None, 8))
    a.submit(enc["pods"])
    ea = full_run_digest.check_engine_run(a, g, "c5 sharded x8")
    a.close()
    b = make_engine(tr, enc, MODE)
    b.submit(enc["pods"])
    eb = full_run_digest.check_engine_run(b, g, "c5 unsharded")
    np.testing.assert_array_equal(ea, eb)
    m = tr["pods"]["m"]
    taint = enc["taint"].astype(np.uint64)
    label = enc["label"].astype(np.uint64)
    tol = enc["pods"]["tol"].astype(np.uint64)
    sel = enc["pods"]["sel"].astype(np.uint64)
    np.testing.assert_array_equal(eb["pod"], np.arange(m))
    assert (np.diff(eb["tick"]) > 0).all() and (eb["status"] == 0).all()
    nd, pods = eb["node"], eb["pod"]
    assert ((taint[nd] & ~tol[pods]) == 0).all()
    assert ((label[nd] & sel[pods]) == sel[pods]).all()
    u, alloc = b.usage(), enc["alloc"]
    for k in range(3):
        has = alloc[:, k] >= 0
        assert (u[has, k] <= alloc[has, k]).all(), f"resource {k} over capacity"


@pytest.mark.parametrize("s0", [167_117, 167_120, 167_127, 166_989, 167_053, 167_128])
def test_c5_segment_overflow_row_on_either_lane_half(c5, s0):
    """Regression test of the round-6 chunk-resolver fix (ks_chunk.hip phase C).
    A batch forced to start at s0 (ks_step(s0), then the rest: a step's first batch starts at its
    first pod) puts pods 167,117 .. 167,180 in one 64-pod chunk in which node 46 changes state six
    times before pod 167,180 (a window expiry, three binds, a second window expiry) — more than the
    five state segments a row holds, so the row's state is unknown for pod 167,180 and the batch must
    stop before it.  The row sits on a lane of the other half of the pod's 16-lane group, whose
    stop flag the old divergent ballot dropped: pod 167,180 then took node 84 instead of node 46
    (both total 18; 46 is the lower index).  Window 10 of the C5 golden (pods 163,840 .. 180,223)
    bind-for-bind against the oracle's digest, with the first ten windows as the run's prefix.
    (s0 = 167,128 is the alignment that never overflowed: the first expiry becomes a head expiry.)"""
    tr, enc = c5
    g = full_run_digest.load("c5")
    if g is None:
        pytest.skip("no c5 golden")
    W = g["window"]
    eng = make_engine(tr, enc, MODE)
    eng.submit(enc["pods"])
    done = 0
    w = 0
    while done + W <= s0:
        b = eng.step(W)
        assert full_run_digest.bind_digest(b) == g["bind_digests"][w], f"window {w}"
        done += W
        w += 1
    parts = [eng.step(s0 - done)] if s0 > done else []
    parts.append(eng.step(done + W - s0))
    b = np.concatenate(parts)
    assert len(b) == W and int(b["pod"][0]) == done
    assert full_run_digest.bind_digest(b) == g["bind_digests"][w], f"window {w} with a batch forced to start at {s0}"


@pytest.mark.parametrize("batch", list(range(128, 257, 16)) + [132, 188, 196, 252])
def test_c5_whole_trace_at_other_batch_sizes(c5, batch):
    """The whole C5 run against the oracle's digests at other batch sizes: each moves every batch
    and chunk boundary, so the chunk resolver's alignment-dependent stops (segment overflow,
    exhausted or truncated lists, slot cuts) fall on other pods (round 6: the lost stop flag above
    showed under 33 of 192 alignments of one batch)."""
    tr, enc = c5
    g = full_run_digest.load("c5")
    if g is None:
        pytest.skip("no c5 golden")
    eng = make_engine(tr, enc, MODE, batch_pods=batch)
    eng.submit(enc["pods"])
    full_run_digest.check_engine_run(eng, g, f"c5 batch {batch}")
