"""Node sharding exchange on CPU with gloo, world_size 2.

Each rank evaluates pods against its node shard only (the oracle's Filter+Score,
oracle/ks_oracle.c ko_eval), keeps the exact per-pod top-L packed keys, the lists are
all-gathered, and the merge must equal the global top-L — whose head is the oracle's bind.
This is the algorithm the device runs (ks_engine.cpp ks_step: per-shard merge, RCCL
all-gather, merge); the GPU suite checks the device path itself (tests/test_engine_gpu.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from harness import make_oracle, small_trace
from kubesim_amd import shard

MODE = "feeds_all_lrba"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, n_nodes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = small_trace(31, n_nodes=n_nodes, n_pods=400, selectors=False)
        ora = make_oracle(tr, MODE)
        ora.submit(tr)
        b, rc = ora.step(150)  # a non-trivial cluster state: pods running, some expired
        assert rc == 0, rc
        lo, hi = shard.rank_nodes(n_nodes, world, rank)
        pods = list(range(150, 182))  # the next pods in FIFO order
        mine = np.zeros((len(pods), shard.TOP_L), np.uint64)
        full = []
        for i, p in enumerate(pods):
            feas, score = ora.eval(p)
            keys = shard.packed_keys(score, (feas != 0) & (score >= 0))
            full.append(shard.top_l(keys))
            if hi > lo:
                mine[i] = shard.top_l(shard.packed_keys(score[lo:hi], (feas[lo:hi] != 0) & (score[lo:hi] >= 0), lo))
        t = torch.from_numpy(mine.view(np.int64).copy())
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        merged = shard.merge_lists(np.stack([x.numpy().view(np.uint64) for x in parts]))
        ok = np.array_equal(merged, np.stack(full))
        # the head of the merged list is the oracle's next bind
        nb, rc = ora.step(1)
        head_node = 0xFFFFFFFF - int(merged[0, 0] & np.uint64(0xFFFFFFFF))
        q.put((rank, bool(ok), rc, int(nb["node"][0]) if len(nb["node"]) else -1, head_node, lo, hi))
    except BaseException as e:  # report instead of leaving the parent waiting
        q.put((rank, False, repr(e), -1, -2, -1, -1))
        raise
    finally:
        dist.destroy_process_group()


def _rank_main_layout(rank, world, vsh, port, n_nodes, q):
    """The exchange in the engine's own layout (ks_shard_layout + ks_step): this rank's vsh parts'
    per-pod top-L lists as its contiguous slice of cand_all[G][B][L], one all-gather, then the
    engine's second merge (ks_merge_candidates, the device merge's per-list step) over the G parts
    of each pod, equal to the global top-L."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G = world * vsh
        pb = shard.engine_part_blocks(n_nodes, world, vsh)   # the engine's geometry, not a restatement
        tr = small_trace(37, n_nodes=n_nodes, n_pods=300, selectors=False)
        ora = make_oracle(tr, MODE)
        ora.submit(tr)
        b, rc = ora.step(100)
        assert rc == 0, rc
        pods = list(range(100, 120))
        B = len(pods)
        mine = np.zeros((vsh, B, shard.TOP_L), np.uint64)   # cand_all[rank*vsh : (rank+1)*vsh]
        full = []
        for i, p in enumerate(pods):
            feas, score = ora.eval(p)
            cand = (feas != 0) & (score >= 0)
            full.append(shard.top_l(shard.packed_keys(score, cand)))
            for v in range(vsh):
                part = rank * vsh + v
                lo = min(int(pb[part]) * shard.BLOCK_NODES, n_nodes)
                hi = min(int(pb[part + 1]) * shard.BLOCK_NODES, n_nodes)
                if hi > lo:
                    mine[v, i] = shard.top_l(shard.packed_keys(score[lo:hi], cand[lo:hi], lo))
        t = torch.from_numpy(mine.reshape(-1).view(np.int64).copy())
        out = torch.zeros(world * t.numel(), dtype=torch.int64)
        dist.all_gather_into_tensor(out, t)
        cand_all = out.numpy().view(np.uint64).reshape(G, B, shard.TOP_L)
        merged = shard.engine_merge(cand_all)  # the engine's own second-merge step
        ok = (np.array_equal(merged, np.stack(full)) and np.array_equal(merged, shard.merge_lists(cand_all))
              and np.array_equal(pb, shard.part_blocks(n_nodes, world, vsh)))
        q.put((rank, bool(ok), 0))
    except BaseException as e:
        q.put((rank, False, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_nodes,vsh", [(1500, 2), (4100, 3), (700, 2)])
def test_shard_exchange_engine_layout_gloo_world2(n_nodes, vsh):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main_layout, args=(r, world, vsh, port, n_nodes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, err in res:
        assert ok, f"rank {rank}: {err or 'merged lists differ from the global top-L'}"


@pytest.mark.parametrize("n_nodes", [300, 1024, 1500])
def test_shard_exchange_gloo_world2(n_nodes):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n_nodes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ranges = [(r[5], r[6]) for r in res]
    assert ranges[0][0] == 0 and ranges[-1][1] == n_nodes and ranges[0][1] == ranges[1][0]
    for rank, ok, rc, bind_node, head_node, lo, hi in res:
        assert ok, f"rank {rank}: merged shard lists differ from the global top-L"
        assert rc == 0 and bind_node == head_node


def test_engine_layout_matches_restatement():
    for n, w, v in ((50_000, 8, 1), (1 << 20, 8, 1), (1000, 4, 1), (100, 4, 1), (4100, 2, 3), (0, 1, 1)):
        np.testing.assert_array_equal(shard.engine_part_blocks(n, w, v), shard.part_blocks(n, w, v))


def test_part_blocks_match_engine_geometry():
    # ks_load_nodes: n_pad = max(64, ceil64(n)); nblk = ceil(n_pad / 256); part p = p * nblk / G
    pb = shard.part_blocks(50_000, 8, 1)
    assert pb[0] == 0 and pb[-1] == (50_048 + 255) // 256 and np.all(np.diff(pb) >= 24)
    assert shard.rank_nodes(1000, 4, 3) == (768, 1000)
    assert shard.rank_nodes(100, 4, 0) == (0, 0)  # one block: parts 0..2 empty


def test_engine_merge_candidates_random():
    """ks_merge_candidates (the device merge's per-list step on the host) against a sort of the
    union, on random sorted 0-padded lists with distinct keys, including empty parts."""
    rng = np.random.default_rng(7)
    for G, B in ((1, 5), (3, 17), (8, 64), (16, 3)):
        keys = np.unique(rng.integers(1, 1 << 40, size=2 * G * B * shard.TOP_L, dtype=np.uint64))
        keys = rng.permutation(keys)[:G * B * shard.TOP_L]
        cand = np.sort(keys.reshape(G, B, shard.TOP_L), axis=2)[:, :, ::-1].copy()
        # ragged: some lists shorter (zero tails), some parts empty for a pod
        cut = rng.integers(0, shard.TOP_L + 1, size=(G, B))
        for g in range(G):
            for b in range(B):
                cand[g, b, cut[g, b]:] = 0
        want = np.zeros((B, shard.TOP_L), np.uint64)
        for b in range(B):
            u = np.sort(cand[:, b, :].ravel())[::-1]
            want[b] = u[:shard.TOP_L]
        np.testing.assert_array_equal(shard.engine_merge(cand), want)

