"""Diagnostic: pair-resolver phase breakdown (s_memtime stamps build, `make stamps`) on the C3
bench workload.  Layout (ks_pair.hip, KS_STAMPS): ctr[8 + 6 * role + i], role 0 walker (wave 0),
1 bind wave (wave 1), 2 owner wave 2, 3 owner wave 7; i 0 work, 1 barrier wait, 2 decision,
3-5 role segments (walker, bind wave); ctr[20..31] work of owner waves 2..13; ctr[5] launches,
ctr[6] pods committed, ctr[7] extra fold rounds."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib
_lib.LIB_PATH = os.path.join(ROOT, "kubernetes-simulator_amd", "kubesim_amd", os.environ.get("KS_DIAG_LIB", "libks_engine_stamps.so"))
from kubesim_amd import tracegen, encode
from kubesim_amd.engine import Engine
tr = tracegen.c3_trace(n_pods=200_000)
enc = encode.encode_trace(tr)
eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)))
eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
eng.submit(enc["pods"])
eng.set_profiling(True)
eng.step(65536)
c0 = eng.debug_counters().copy()
t = time.perf_counter(); eng.step(32768); dt = time.perf_counter() - t
st = eng.last_step_stats()
d = eng.debug_counters() - c0
pods, L = max(d[6], 1), max(d[5], 1)
pairs = pods / 2
print(f"pods={pods} launches={L} ({pods / L:.1f} pods/launch) wall {dt * 1e3:.1f} ms -> {32768 / dt:.0f} pods/s")
seg = {0: ("K2 of c", "stage + fold", "walk"), 1: ("expiry scan", "fetch + binds", "eval + fold")}
for role, name in ((0, "walker"), (1, "bind wave")):
    b = 8 + 6 * role
    print(f"{name:13s} work {d[b] / pairs:7.0f}  wait {d[b + 1] / pairs:6.0f}  decision {d[b + 2] / pairs:5.0f}  " +
          "  ".join(f"{seg[role][i]} {d[b + 3 + i] / pairs:5.0f}" for i in range(3)) + "  cycles/pair")
print("owner waves 2..13 work (cycles/pair, 0 = ended early): " +
      " ".join(f"{d[20 + w] / pairs:.0f}" for w in range(12)))
print(f"extra fold rounds: {d[7] / L:.2f} per launch ({d[7] / pairs * 100:.2f} % of pairs)")
nl = max(st["launches"], 1)
print(f"resolve {st['resolve_ms'] / nl * 1e3:.1f} us/launch, scan {st['scan_ms'] / nl * 1e3:.1f}, other {st['other_ms'] / nl * 1e3:.1f}; "
      f"resolve {st['resolve_ms'] * 1e6 / max(st['pods'], 1):.0f} ns/pod")
