"""Diagnostic A/B of the scan kernel across engine builds (GPU box; timing only):
    python tests/dev/ab_scan.py libks_engine_A.so [C3|C5]
prints the profiled per-launch scan / resolve / other ms of a few C3 or C5 batches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402

_lib.LIB_PATH = lib_path(sys.argv[1])
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402

cfg = sys.argv[2] if len(sys.argv) > 2 else "C5"
tr = tracegen.c5_trace(n_pods=12_000) if cfg == "C5" else tracegen.c3_trace(n_pods=40_000)
enc = encode.encode_trace(tr)
eng = Engine(tick_seconds=tr["tick_seconds"], filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)))
eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
eng.submit(enc["pods"])
eng.step(2048)
eng.set_profiling(True)
b = eng.step(8192)
import zlib  # noqa: E402
crc = zlib.crc32(b["node"].tobytes() + b["status"].tobytes())
st = eng.last_step_stats()
n = max(st["launches"], 1)
print(f"{sys.argv[1]} {cfg}: scan {st['scan_ms'] / n * 1e3:.1f} us  resolve {st['resolve_ms'] / n * 1e3:.1f} us  "
      f"other {st['other_ms'] / n * 1e3:.1f} us  launches {n}  binds {len(b)} crc {crc:08x}", flush=True)
