"""Diagnostic: resolver phase breakdown (s_memtime stamps build) on the C3 bench workload."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib
_lib.LIB_PATH = lib_path(os.environ.get("KS_DIAG_LIB", "libks_engine_stamps.so"))
from kubesim_amd import tracegen, encode
from kubesim_amd.engine import Engine
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
tr = tracegen.c3_trace(n_pods=200_000)
enc = encode.encode_trace(tr)
eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), batch_pods=B)
eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
eng.submit(enc["pods"])
from kubesim_amd.engine import KsError
def step(n):
    try:
        eng.step(n)
    except KsError as ex:  # ablation builds (timing only) may stop early
        print("  stopped:", ex)
eng.set_profiling(True)
step(65536)
st0 = eng.last_step_stats()
nl0 = max(st0["launches"], 1)
print(f"  warmup: resolve {st0['resolve_ms'] * 1e6 / max(st0['pods'], 1):.0f} ns/pod, {st0['pods'] / nl0:.1f} pods/launch")
c0 = eng.debug_counters().copy()
eng.set_profiling(True)
t = time.perf_counter(); step(32768); dt = time.perf_counter() - t
st = eng.last_step_stats()
c1 = eng.debug_counters()
d = c1 - c0
D = d[16:]
pods = D[4]
print(f"B={B} pods={st['pods']} wall {dt*1e3:.1f} ms  -> {32768/dt:.0f} pods/s")
# layout (ks_kernels.hip, KS_STAMPS): D = ctr[16..31]; D[0]/D[1] wave 0 work / barrier wait,
# D[2] wave 1 work, D[3] wave 2 work, D[15] wave 3 (first owner) work; D[5..8] wave 3 segments
# (top, load, exclusion, eval); D[11..14] wave 1 segments (fetch+fit, expiries, -, eval);
# ctr[5..7] wave 0 segments (insert, commit, issue); D[9] owner lanes past the prune, D[10] owner
# waves evaluating
for k, name in ((0, "w0 work"), (1, "w0 wait"), (2, "w1 work"), (3, "w2 work"), (15, "w3 work"),
                (5, "w3 top"), (6, "w3 load"), (7, "w3 excl"), (8, "w3 eval"),
                (11, "w1 fetch+fit"), (12, "w1 expiries"), (14, "w1 eval")):
    print(f"  {name:12s} {D[k]/max(pods,1):9.0f} cycles/pod")
for k, name in ((5, "w0 insert"), (6, "w0 commit"), (7, "w0 issue")):
    print(f"  {name:12s} {d[k]/max(pods,1):9.0f} cycles/pod")
for k, name in ((9, "owner lanes"), (10, "owner waves")):
    print(f"  {name:12s} {D[k]/max(pods,1):9.2f} per pod")
L = max(d[14] or st["launches"], 1)
print(f"  launches {d[14]}  pods/launch {pods / L:.1f}  expiries/launch {d[15] / L:.1f}")
for k, name in ((8, "init+search"), (9, "loads"), (10, "pre-insert"), (11, "table loads"), (12, "prologue"), (13, "writeback")):
    print(f"  {name:12s} {d[k] / L:9.0f} cycles/launch")
nl = max(st["launches"], 1)
print(f"  resolve {st['resolve_ms'] / nl * 1e3:.1f} us/launch, scan {st['scan_ms'] / nl * 1e3:.1f}, other {st['other_ms'] / nl * 1e3:.1f}; "
      f"{st['pods'] / nl:.1f} pods/launch, resolve {st['resolve_ms'] * 1e6 / max(st['pods'], 1):.0f} ns/pod")
loop = (D[0] + D[1]) / L
setup = sum(d[k] for k in (8, 9, 10, 11, 12, 13)) / L
print(f"  stamp clock ~ {(loop + setup) / (st['resolve_ms'] / L * 1e3) / 1e3:.2f} GHz (loop+setup cycles / resolve time)")
