"""Every resolver against the oracle (kubesim/kubesim.go:90-225 restated in oracle/ks_oracle.c).

The engine has exact resolvers for step 4 of a batch: the role-split one-pod
kernel, the register-table kernel (small clusters) and the chunk kernel (chunked Jacobi sweeps in
one workgroup's LDS, over the candidate lists of ks_cand.hip).  The engine picks one
by size class; the KS_ENGINE_*_RESOLVER flags force one, and each forced resolver must give the
oracle's binds, statuses and usage on every case below — all filter / scorer modes, batch sizes
from 3 to 256, dense in-batch expiries, forced list exhaustion, and a C2 prefix.
"""
import numpy as np
import pytest

from harness import MODES, assert_same_binds, encoded, engine_run, make_engine, make_oracle, oracle_run, small_trace
from kubesim_amd import _lib, tracegen

pytestmark = pytest.mark.gpu
RESOLVERS = {"one_pod": _lib.KS_ENGINE_ONE_POD_RESOLVER, "chunk": _lib.KS_ENGINE_CHUNK_RESOLVER,
             # the chunk resolver on pruned block lists (ks_scan.h: a block writes only keys that can
             # reach the pod's global top-L; the merge reads the flagged blocks)
             "chunk_pruned": _lib.KS_ENGINE_CHUNK_RESOLVER | _lib.KS_ENGINE_PRUNED_LISTS}


def _run(tr, mode, ticks, batch, flags, chunks):
    enc = encoded(tr)
    eng = make_engine(tr, enc, mode, batch, flags)
    eng.submit(enc["pods"])
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    left = ticks
    for c in chunks:
        k = min(c, left)
        if k <= 0:
            break
        eb, erc = engine_run(eng, k, k)
        ob, orc = oracle_run(ora, k)
        assert_same_binds(eb, ob)
        assert erc == orc, (erc, orc)
        left -= k
        if erc:
            return eng
        np.testing.assert_array_equal(eng.usage(), ora.usage())
    return eng


@pytest.mark.parametrize("res", sorted(RESOLVERS))
@pytest.mark.parametrize("mode", sorted(MODES))
def test_modes(res, mode):
    tr = small_trace(1, n_nodes=400, n_pods=600, arrival="stream")
    _run(tr, mode, 800, 256, RESOLVERS[res], (1, 7, 100, 692))


@pytest.mark.parametrize("res", sorted(RESOLVERS))
@pytest.mark.parametrize("batch", [3, 64, 256])
def test_batches(res, batch):
    tr = small_trace(7, n_nodes=300, n_pods=2500, taints=False, selectors=False)
    _run(tr, "literal_lrba_filters_ignored", 2500, batch, RESOLVERS[res], (1, 17, 500, 1982))


@pytest.mark.parametrize("res", sorted(RESOLVERS))
def test_dense_expiries(res):
    tr = small_trace(11, n_nodes=2000, n_pods=6000, taints=False, selectors=False, tolerations=False)
    p = tr["pods"]
    p["phase_sec"][:] = 1 + (np.arange(len(p["phase_sec"])) % 12)
    _run(tr, "feeds_all_lrba", 6000, 256, RESOLVERS[res], (1500,) * 4)


@pytest.mark.parametrize("res", sorted(RESOLVERS))
def test_list_exhaustion(res):
    tr = small_trace(21, n_nodes=300, n_pods=900, taints=False, labels=False, tolerations=False,
                     selectors=False)
    nd, p = tr["nodes"], tr["pods"]
    p["req"][:] = p["req"][0]
    nd["alloc"][:, :3] = 4 * p["req"][0]
    nd["alloc"][:, 3] = 110
    nd["alloc_has"][:] = 15
    _run(tr, "feeds_fit_lr", 900, 256, RESOLVERS[res], (900,))


@pytest.mark.parametrize("res", sorted(RESOLVERS))
@pytest.mark.parametrize("mode", ["feeds_all_lrba", "literal_lrba_filters_ignored"])
def test_c2_prefix(res, mode):
    tr = tracegen.c2_trace(n_pods=12_000)
    _run(tr, mode, 12_000, 0, RESOLVERS[res], (4096, 7904))


# ---- the chunk resolver on the wide evaluator (32-bit state words, ks_chunk.hip NS32) -----------
@pytest.mark.parametrize("mode", ["feeds_all_lrba", "literal_lrba_filters_ignored"])
def test_chunk_wide_evaluator(mode):
    """FORCE_WIDE on small capacities: the chunk kernel's wide instantiation (widened words, the
    wide evaluator) on the cases above."""
    tr = small_trace(1, n_nodes=400, n_pods=600, arrival="stream")
    _run(tr, mode, 800, 256, RESOLVERS["chunk"] | _lib.KS_ENGINE_FORCE_WIDE, (1, 7, 100, 692))


def test_chunk_decimal_memory_class():
    """Decimal-SI memory requests on binary-SI capacities (C3q's distributions at 2k nodes): the
    gcd scaling leaves memory capacities up to 2^31, beyond int32 — the engine's default picks the
    chunk resolver on uint32 words with the wide evaluator; binds, statuses and usage against the
    oracle, with dense expiries."""
    tr = tracegen.c3q_trace(n_nodes=2000, n_pods=8000)
    assert int(np.max(tr["nodes"]["alloc"][:, 1])) == 512 * (1 << 30) * 1000  # 512Gi: 2^31 after the gcd
    _run(tr, "feeds_all_lrba", 8000, 0, 0, (2500, 5500))


# ---- the overlap (next batch's scan fused into the chunk kernel, ks_engine.cpp step loop) ------
def _engine_env(tr, enc, mode, overlap, engine_flags=0, **kw):
    flags = engine_flags | (0 if overlap else _lib.KS_ENGINE_NO_OVERLAP)
    return make_engine(tr, enc, mode, engine_flags=flags, **kw)


@pytest.mark.parametrize("pruned", [False, True], ids=["full_lists", "pruned_lists"])
@pytest.mark.parametrize("case", ["c2", "dense_expiries"])
def test_overlap_on_and_off_bind_identically_and_match_oracle(case, pruned):
    """The speculative lists (stale for the nodes the previous batch touched, which join E) and
    the conditional rescan after early stops: the overlapped chain gives the plain chain's binds,
    statuses and usage, and the oracle's."""
    if case == "c2":
        tr = tracegen.c2_trace(n_pods=12_000)
        mode, ticks, chunks = "feeds_all_lrba", 12_000, (5000, 7000)
    else:
        tr = small_trace(11, n_nodes=2000, n_pods=6000, taints=False, selectors=False, tolerations=False)
        tr["pods"]["phase_sec"][:] = 1 + (np.arange(len(tr["pods"]["phase_sec"])) % 12)
        mode, ticks, chunks = "feeds_all_lrba", 6000, (1500,) * 4
    enc = encoded(tr)
    ora = make_oracle(tr, mode)
    ora.submit(tr)
    ob, orc = oracle_run(ora, ticks)
    assert orc == 0
    for overlap in (False, True):  # (the chunk resolver forced: these clusters are the small class)
        eng = _engine_env(tr, enc, mode, overlap, batch_pods=192,
                          engine_flags=RESOLVERS["chunk_pruned" if pruned else "chunk"])
        eng.submit(enc["pods"])
        got = []
        for c in chunks:
            eb, erc = engine_run(eng, c, c)
            got.append(eb)
            assert erc == 0
        assert_same_binds(np.concatenate(got), ob)
        np.testing.assert_array_equal(eng.usage(), ora.usage())
        eng.close()
