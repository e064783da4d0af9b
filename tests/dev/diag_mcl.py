"""Diagnostic: merge_cl and window-prep section cycles (`make variant NAME=mcldiag DEFS=-DKS_MCL_DIAG`,
thread 0's s_memtime deltas; the product executes none of it) on the C3 bench workload, overlap on.
ctr[5] merge_cl workgroups, [6..12] their sections (block lists + E keys + inserts, wave merges +
barrier, final merge, candidate e_idx + threshold, E inclusion, ranking, slot claims); [23] window
preps, [16..22] their sections (first loads to the count barrier, head + window loads and hashing,
touched inserts, counts, prefix, slot fill, sort + e_idx + tail)."""
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402
_lib.LIB_PATH = lib_path(os.environ.get("KS_DIAG_LIB", "libks_engine_mcldiag.so"))
from kubesim_amd import tracegen, encode  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402
tr = tracegen.c3_trace(n_pods=200_000)
enc = encode.encode_trace(tr)
eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), engine_flags=64)
eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
eng.submit(enc["pods"])
eng.step(32768)
c0 = eng.debug_counters().copy()
t = time.perf_counter(); eng.step(32768); dt = time.perf_counter() - t
d = eng.debug_counters() - c0
W = max(d[5], 1)
names = ("lists+E keys+inserts", "wave merges+barrier", "final merge", "cand e_idx+thr", "E inclusion", "ranking", "slot claims")
print(f"merge_cl workgroups {W}; cycles per workgroup: " + ", ".join(f"{n} {d[6 + q] / W:.0f}" for q, n in enumerate(names)))
print(f"   total {sum(d[6:13]) / W:.0f}; wall {32768 / dt:.0f} pods/s")
P = max(d[23], 1)
pn = ("loads to count", "head+window loads, hashing", "touched inserts", "counts", "prefix", "slot fill", "sort+e_idx+tail")
print(f"window preps {P}; cycles each: " + ", ".join(f"{n} {d[16 + q] / P:.0f}" for q, n in enumerate(pn)) + f"; total {sum(d[16:23]) / P:.0f}")
if "--d2" in sys.argv:  # (DEFS=-DKS_MCL_DIAG=2: waits inserted, timing shifts)
    print(f"thread 0: to the first reads (counts, pod index, first list) {d[13] / W:.0f}, E chain {d[14] / W:.0f} cycles "
          f"over {d[24] / W:.2f} E nodes; n_e {d[25] / W:.1f}")
