"""The multi-rank sharded device path (VERDICT r3 "what's missing" 2) with ranks as
engines on threads of one process, exchanging candidates through the host (ks_shard_host +
ks_local_allgather) instead of RCCL — RCCL refuses two ranks on one GPU.  Rank r scans only its
blocks [blk_lo, blk_lo + blk_n) and writes its parts' slices of cand_all; the exchange hands every
rank all parts; the second merge and the resolver then give every rank the global argmax of
kubesim/kubesim.go:208-222.  Checked: both ranks bind-for-bind against the oracle (small and C2
sizes, uneven parts) and the whole C5 run against the committed oracle digests."""
import threading

import numpy as np
import pytest

import full_run_digest
from harness import assert_same_binds, encoded, make_engine, make_oracle, small_trace
from kubesim_amd import _lib, shard, tracegen
from kubesim_amd.engine import LocalExchange

pytestmark = pytest.mark.gpu
MODE = "feeds_all_lrba"


def _ranks(tr, enc, world, vshards, mode=MODE, **kw):
    x = LocalExchange(world)
    engs = []
    for r in range(world):
        from kubesim_amd.engine import Engine
        from harness import MODES
        fm, fl, sc = MODES[mode]
        e = Engine(tick_seconds=tr["tick_seconds"], filter_mode=fm, filters=fl, scorers=sc, **kw)
        e.shard_host(world, r, x, vshards)
        e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
        e.submit(enc["pods"])
        engs.append(e)
    return engs, x


def _step_all(engs, k, x=None):
    out = [None] * len(engs)

    def run(r):
        try:
            out[r] = engs[r].step(k)
        except Exception as ex:  # noqa: BLE001 - reported below
            out[r] = ex
            if x is not None:  # the other ranks would wait for this one's deposit
                x.abort()
    th = [threading.Thread(target=run, args=(r,)) for r in range(len(engs))]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    assert not any(t.is_alive() for t in th), "a rank hung in the exchange"
    for o in out:
        if isinstance(o, Exception):
            raise o
    return out


@pytest.mark.parametrize("world,vshards", [(2, 1), (2, 3), (3, 2)])
def test_ranks_match_oracle_small(world, vshards):
    tr = small_trace(3, n_nodes=3000, n_pods=2500, arrival="stream")
    enc = encoded(tr)
    engs, _x = _ranks(tr, enc, world, vshards, batch_pods=128)
    ora = make_oracle(tr, MODE)
    ora.submit(tr)
    for k in (1, 700, 1900):
        bs = _step_all(engs, k, _x)
        ob, rc = ora.step(k, cap=k)
        for b in bs:
            assert_same_binds(b, ob)
        assert rc == 0
    for e in engs:
        np.testing.assert_array_equal(e.usage(), ora.usage())


@pytest.mark.parametrize("flags", [0, _lib.KS_ENGINE_PRUNED_LISTS, _lib.KS_ENGINE_NO_OVERLAP],
                         ids=["overlap", "overlap_pruned", "plain_chain"])
def test_c2_prefix_two_ranks_match_oracle(flags):
    """C2 on the chunk resolver: by default with the overlap (each rank's speculative scan of its
    own blocks fused into its chunk kernel, the exchange every batch), also with pruned lists (the
    per-part merges read only flagged blocks) and on the plain chain."""
    tr = tracegen.c2_trace(n_pods=8000)
    enc = encoded(tr)
    engs, _x = _ranks(tr, enc, 2, 2, engine_flags=flags)
    ora = make_oracle(tr, MODE)
    ora.submit(tr)
    for k in (4096, 3904):
        bs = _step_all(engs, k, _x)
        ob, rc = ora.step(k, cap=k)
        assert rc == 0
        for b in bs:
            assert_same_binds(b, ob)
    for e in engs:
        np.testing.assert_array_equal(e.usage(), ora.usage())


def test_c5_whole_trace_two_ranks_match_oracle_golden():
    """BASELINE configs[4] as 2 ranks x 4 parts (the 8 parts of the 8-GPU layout): every pod the
    bench's C5 leg binds, window by window against tests/golden/full_run.json on both ranks."""
    g = full_run_digest.load("c5")
    if g is None:
        pytest.skip("no c5 golden")
    tr = tracegen.c5_trace(n_pods=g["pods"])
    enc = encoded(tr)
    assert g["nodes"] == tr["nodes"]["n"]
    engs, _x = _ranks(tr, enc, 2, 4)
    done = 0
    for w, want in enumerate(g["bind_digests"]):
        k = min(g["window"], g["pods"] - done)
        bs = _step_all(engs, k, _x)
        for r, b in enumerate(bs):
            assert len(b) == k and int(b["pod"][0]) == done
            assert full_run_digest.bind_digest(b) == want, f"rank {r}: window {w} differs"
        done += k


def _c5_golden_ranks(world, **kw):
    """Every pod of the C5 leg on `world` thread-ranks (one part each) against the committed oracle
    digests, window by window on every rank, with the between-step invariants of every rank's
    engine (ks_debug_invariants: no candidate-slot or E-index mark left set).  Returns the largest
    number of candidate slots a batch claimed on any rank."""
    g = full_run_digest.load("c5")
    if g is None:
        pytest.skip("no c5 golden")
    tr = tracegen.c5_trace(n_pods=g["pods"])
    enc = encoded(tr)
    engs, _x = _ranks(tr, enc, world, 1, **kw)
    done = 0
    hw = 0
    for w, want in enumerate(g["bind_digests"]):
        k = min(g["window"], g["pods"] - done)
        bs = _step_all(engs, k, _x)
        for r, b in enumerate(bs):
            assert len(b) == k and int(b["pod"][0]) == done
            assert full_run_digest.bind_digest(b) == want, f"rank {r}: window {w} differs"
            inv = engs[r].debug_invariants()
            assert inv["slot_marks"] == 0 and inv["e_marks"] == 0, (r, w, inv)
            hw = max(hw, inv["nslot_hw"])
        done += k
    return hw


def test_c5_whole_trace_sixteen_ranks_overlapped_match_oracle_golden():
    """BASELINE configs[4] as 16 ranks: 256 scan blocks per rank, so every rank runs the overlap
    (its speculative scan fused into its chunk kernel; ks_engine.cpp kOverlapMaxBlocks) on pruned
    lists (1M nodes), with the exchange every batch — every pod of the C5 leg against
    tests/golden/full_run.json on every rank."""
    _c5_golden_ranks(16)


def test_c5_whole_trace_eight_ranks_deployment_layout_match_oracle_golden():
    """BASELINE configs[4] in the 8-GPU deployment layout: 8 thread-ranks x 1 part, 512 scan blocks
    per rank — above kOverlapMaxBlocks, so every rank runs the plain chain on pruned lists (1M
    nodes) with the exchange every batch; every pod against tests/golden/full_run.json on every
    rank."""
    _c5_golden_ranks(8)


def test_ranks_without_scan_blocks_match_oracle():
    """A chunk-resolver cluster smaller than its shard layout: 600 nodes = 3 scan blocks
    over 4 ranks, so rank 0 scans nothing and its scan launch only stages the batch's E records for
    merge_cl (ks_kernels.hip scan_kernel).  Every rank bind-for-bind against the oracle, up to the
    same aborting error (a 600-node cluster leaves some selector pairs on no node: NotFound,
    kubesim/kubesim.go:217-220, exactly where the oracle stops)."""
    from kubesim_amd.engine import KsError
    tr = small_trace(11, n_nodes=600, n_pods=1500, arrival="stream")
    enc = encoded(tr)
    assert 0 in np.diff(shard.engine_part_blocks(600, 4)), "a rank without scan blocks"
    world = 4
    engs, x = _ranks(tr, enc, world, 1, batch_pods=64, engine_flags=_lib.KS_ENGINE_CHUNK_RESOLVER)
    ora = make_oracle(tr, MODE)
    ora.submit(tr)
    ob, orc = ora.step(1500, cap=1500)
    out = [None] * world

    def run(r):
        try:
            out[r] = (engs[r].step(1500), 0)
        except KsError as ex:
            out[r] = (ex.binds, ex.code)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    assert not any(t.is_alive() for t in th), "a rank hung in the exchange"
    for b, code in out:
        assert code == orc
        assert_same_binds(b, ob)
    for e in engs:
        np.testing.assert_array_equal(e.usage(), ora.usage())
        inv = e.debug_invariants()
        assert inv["slot_marks"] == 0 and inv["e_marks"] == 0, inv
