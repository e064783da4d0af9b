"""Dev tool (not a test): per-kernel HIP-event times (ks_last_step_kernels) of the C3 bench workload
with the overlap on and off, on one engine build (KS_LIB, devlib.lib_path), plus the debug counters'
early stops.  usage: python tests/dev/kernel_ab.py [--pods 65536] [--c5]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402
_lib.LIB_PATH = lib_path(os.environ.get("KS_LIB", "libks_engine.so"))
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402

c5 = "--c5" in sys.argv
S = 32768
tr = tracegen.c5_trace(n_pods=5 * S) if c5 else tracegen.c3_trace(n_pods=5 * S)
enc = encode.encode_trace(tr)
for flags in (0, _lib.KS_ENGINE_NO_OVERLAP):
    eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), engine_flags=flags)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    eng.submit(enc["pods"])
    eng.step(S)
    c0 = eng.debug_counters().copy()
    t = time.perf_counter()
    eng.step(S)
    dt = time.perf_counter() - t
    eng.set_profiling(True)
    eng.step(S)
    st, k = eng.last_step_stats(), eng.last_step_kernels()
    d = eng.debug_counters() - c0
    nb = max(st["launches"], 1)
    per = {r: (k[r + "_ms"] / max(k[r + "_n"], 1) * 1e3, k[r + "_n"] / nb) for r in ("prep", "scan", "merge", "resolve", "fused")}
    print(f"{'plain' if flags else 'overlap'}: {S / dt:.0f} pods/s wall, {st['step_ms'] / nb * 1e3:.1f} us per batch "
          f"(profiled), {st['pods'] / nb:.1f} pods/batch, early stops {int(d[4])} / {nb * 2}")
    print("   " + ", ".join(f"{r} {v[0]:.1f} us x {v[1]:.2f}" for r, v in per.items()))
    eng.close()
