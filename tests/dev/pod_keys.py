"""Dev tool (not a test): the exact scores of one pod of the C5 trace after the pods before it are
bound (unsharded engine, ks_step + ks_score at the current tick) — for a bind that differs between
two builds (tests/dev/byval_diag.py).  python tests/dev/pod_keys.py POD NODE..."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402
_lib.LIB_PATH = lib_path(os.environ.get("KS_LIB", "libks_engine.so"))
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402

P = int(sys.argv[1])
nodes = [int(x) for x in sys.argv[2:]]
tr = tracegen.c5_trace(n_pods=196608)
enc = encode.encode_trace(tr)
e = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)))
e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
e.submit(enc["pods"])
b = e.step(P)
print("tick", e.tick, "binds", len(b))
sc = e.score(P)
order = np.lexsort((np.arange(len(sc)), -sc))
print("top 24 (node, total):", [(int(n), int(sc[n])) for n in order[:24]])
for n in nodes:
    print(f"node {n}: total {int(sc[n])}, rank {int(np.nonzero(order == n)[0][0])}, alloc {enc['alloc'][n].tolist()}")
u = e.usage()
for n in nodes:
    print(f"node {n}: usage {u[n].tolist()}")
nb = e.step(1)
print("bind of pod", P, nb)
