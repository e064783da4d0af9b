"""Per-tick drop-in rate on the C3 cluster (one arrival per tick): the C++ Run loop (NativeRun)
per tick and windowed — bench.py's dropin leg, alone."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
sys.path.insert(0, ROOT)
import bench
from kubesim_amd import encode, tracegen
tr = tracegen.c3_trace(n_pods=80_000)
enc = encode.encode_trace(tr)
t = time.perf_counter()
out = bench.dropin_leg(tr, enc, ((1, 1, 0), (2, 1, 0)), 0)
for k, v in out.items():
    print(k, v)
