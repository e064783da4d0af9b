"""Diagnostic: share of the scan kernel's wave-0 cycles in evaluation (phase 1) and top-L
extraction (phase 2): build with make variant NAME=sst DEFS=-DKS_SCAN_STAMPS."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402

_lib.LIB_PATH = lib_path("libks_engine_sst.so")
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402

for cfg in ("C3", "C5"):
    tr = tracegen.c5_trace(n_pods=12_000) if cfg == "C5" else tracegen.c3_trace(n_pods=40_000)
    enc = encode.encode_trace(tr)
    eng = Engine(tick_seconds=tr["tick_seconds"], filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)))
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    eng.submit(enc["pods"])
    eng.step(2048)
    c0 = eng.debug_counters().copy()
    eng.step(8192)
    d = eng.debug_counters() - c0
    tot = max(int(d[20] + d[21]), 1)
    print(f"{cfg}: evaluation {d[20] / tot:.2f}, top-L extraction {d[21] / tot:.2f} of wave-0 cycles", flush=True)
    eng.close()
