"""Diagnostic: phase breakdown of the register-table resolver (ks_resolve.hip built with
-DKS_R4_STAMPS: make -C kubernetes-simulator_amd/csrc variant NAME=st DEFS=-DKS_R4_STAMPS) on one
C4 what-if scenario (2,000 nodes, 128-pod batches: the small class it serves).  Stamps wait for
LDS (s_waitcnt lgkmcnt(0)), so phases are serialised a little."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402

_lib.LIB_PATH = lib_path(sys.argv[1] if len(sys.argv) > 1 else "libks_engine_st.so")
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402

tr = tracegen.c4_scenario(0, n_nodes=2000, n_pods=40_000)
enc = encode.encode_trace(tr)
eng = Engine(tick_seconds=tr["tick_seconds"], filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)))
eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
eng.submit(enc["pods"])
eng.step(4096)
c0 = eng.debug_counters().copy()
eng.set_profiling(True)
t = time.perf_counter()
eng.step(8192)
dt = time.perf_counter() - t
st = eng.last_step_stats()
d = eng.debug_counters() - c0
it, L = max(int(d[5]), 1), max(int(d[6]), 1)
names = ("decide", "bind", "expiries", "mask", "eval", "barrier")
print(f"{8192 / dt:.0f} pods/s; resolve {st['resolve_ms'] * 1e6 / max(st['pods'], 1):.0f} ns/pod; "
      f"{it / L:.1f} pods/launch")
for w in range(4):
    row = [d[8 + 6 * w + k] / it for k in range(6)]
    print(f"  wave {w}: " + "  ".join(f"{n} {v:6.0f}" for n, v in zip(names, row)) + f"  total {sum(row):6.0f} cycles/pod")
