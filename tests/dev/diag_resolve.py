"""Diagnostic: resolver phase breakdown (s_memtime stamps build) on the C3 bench workload."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib
_lib.LIB_PATH = os.path.join(ROOT, "kubernetes-simulator_amd", "kubesim_amd", "libks_engine_stamps.so")
from kubesim_amd import tracegen, encode
from kubesim_amd.engine import Engine
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
tr = tracegen.c3_trace(n_pods=200_000)
enc = encode.encode_trace(tr)
eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), batch_pods=B)
eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
eng.submit(enc["pods"])
eng.step(65536)
c0 = eng.debug_counters().copy()
t = time.perf_counter(); eng.step(32768); dt = time.perf_counter() - t
c1 = eng.debug_counters()
d = c1 - c0
pods = d[12]
print(f"B={B} pods={pods} wall {dt*1e3:.1f} ms  -> {32768/dt:.0f} pods/s")
for k, name in enumerate(["wave0 work", "wave0 wait", "wave1 work", "wave3 work"]):
    print(f"  {name:11s} {d[8+k]/max(pods,1):9.0f} cycles/pod")
for k, name in ((7, "w3 winner"), (13, "w3 excl+ld"), (14, "w3 eval"), (15, "w3 reduce")):
    print(f"  {name:11s} {d[k]/max(pods,1):9.0f} cycles/pod")
