"""Dev tool (not a test): VERDICT r5 item 1 — the C5 leg on thread-ranks (ks_shard_host), window by
window against the committed oracle digests, with every rank's binds saved and compared with each
other, so a diagnostic build (KS_LIB, tests/dev/devlib.py; e.g. the by-value merge_cl of commit
63524d5: make -C kubernetes-simulator_amd/csrc variant NAME=byval DEFS=-DKS_MCL_BYVAL) can be
compared bind for bind with the product.

    python tests/dev/byval_diag.py WORLD [FLAGS] OUT.npz"""
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402
_lib.LIB_PATH = lib_path(os.environ.get("KS_LIB", "libks_engine.so"))
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine, LocalExchange  # noqa: E402
import full_run_digest  # noqa: E402

world = int(sys.argv[1])
flags = int(sys.argv[2]) if len(sys.argv) > 2 else 0
out = sys.argv[3] if len(sys.argv) > 3 else None
g = full_run_digest.load("c5")
tr = tracegen.c5_trace(n_pods=g["pods"])
enc = encode.encode_trace(tr)
x = LocalExchange(world) if world > 1 else None
es = []
for r in range(world):
    e = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), engine_flags=flags)
    if world > 1:
        e.shard_host(world, r, x, 1)
    e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    e.submit(enc["pods"])
    es.append(e)
done = 0
nodes, stats = [], []
first_bad = None
for w, want in enumerate(g["bind_digests"]):
    k = min(g["window"], g["pods"] - done)
    res = [None] * world
    th = [threading.Thread(target=lambda r=r: res.__setitem__(r, es[r].step(k))) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    ok = [full_run_digest.bind_digest(b) == want for b in res]
    same = all(np.array_equal(res[0]["node"], b["node"]) and np.array_equal(res[0]["status"], b["status"]) for b in res)
    early = int(es[0].debug_counters()[4])
    inv = es[0].debug_invariants()
    print(f"window {w}: golden ok on ranks {sum(ok)}/{world}; ranks identical {same}; early stops {early}; {inv}", flush=True)
    if not same:
        for r in range(1, world):
            d = np.nonzero((res[0]["node"] != res[r]["node"]) | (res[0]["status"] != res[r]["status"]))[0]
            if len(d):
                print(f"   rank {r} differs from rank 0 first at pod {done + int(d[0])}", flush=True)
    if first_bad is None and not all(ok):
        first_bad = w
    nodes.append(np.stack([b["node"] for b in res]))
    stats.append(np.stack([b["status"] for b in res]))
    done += k
if out:
    np.savez_compressed(out, nodes=np.concatenate(nodes, axis=1), status=np.concatenate(stats, axis=1))
print(f"first window off the golden: {first_bad}")
