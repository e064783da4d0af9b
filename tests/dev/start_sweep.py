"""Dev tool (not a test): the C5 trace with the chunk resolver's first batch forced to start at each
pod s0 of a range (ks_step(s0), then ks_step(n): a step's first batch starts at its first pod), each
window of n pods compared bind for bind with known-correct binds (build/diag/c5_truth.npz, from a
run that matches the oracle's golden digests) — to find a batch alignment under which a bind comes
out wrong.  python tests/dev/start_sweep.py LO HI N [FLAGS]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import DIAG, lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402
_lib.LIB_PATH = lib_path(os.environ.get("KS_LIB", "libks_engine.so"))
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402

from winws import show_watch  # noqa: E402

lo, hi, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
WATCH = int(os.environ.get("WATCH", "-1"))
NODES = [int(x) for x in os.environ.get("WATCH_NODES", "").split(",") if x]
flags = int(sys.argv[4]) if len(sys.argv) > 4 else 0
truth = np.load(os.path.join(DIAG, "c5_truth.npz"))
tr = tracegen.c5_trace(n_pods=196608)
enc = encode.encode_trace(tr)
bad = 0
for s0 in range(lo, hi):
    e = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), engine_flags=flags)
    e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    e.submit(enc["pods"])
    e.step(s0)
    if WATCH >= 0:
        e.debug_watch(WATCH)
    b = e.step(n)
    if WATCH >= 0:
        show_watch(e, WATCH, NODES)
    d = np.nonzero((b["node"] != truth["node"][s0:s0 + n]) | (b["status"] != truth["status"][s0:s0 + n]))[0]
    if len(d):
        bad += 1
        p = s0 + int(d[0])
        print(f"s0 {s0}: first wrong bind pod {p}: node {int(b['node'][d[0]])} (truth {int(truth['node'][p])}); "
              f"{len(d)} wrong of {n}", flush=True)
    e.close()
    if s0 % 16 == 0:
        print(f"... s0 {s0}", flush=True)
print(f"{bad} of {hi - lo} alignments wrong")
