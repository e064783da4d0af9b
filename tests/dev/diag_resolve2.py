"""Diagnostic: per-wave work cycles per pod of the speculative resolver (KS_STAMPS build,
libks_engine_stamps.so: ctr[16 + wave] = cycles each wave spent between its barriers, ctr[5] = pods)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib
_lib.LIB_PATH = os.path.join(ROOT, "kubernetes-simulator_amd", "kubesim_amd", os.environ.get("KS_DIAG_LIB", "libks_engine_stamps.so"))
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
eng.set_profiling(True)
t = time.perf_counter(); eng.step(32768); dt = time.perf_counter() - t
st = eng.last_step_stats()
d = eng.debug_counters() - c0
pods = max(int(d[5]), 1)
ns = st["resolve_ms"] * 1e6 / max(st["pods"], 1)
print(f"B={B} pods={st['pods']} wall {dt*1e3:.1f} ms; resolve {ns:.0f} ns/pod, {st['pods'] / max(st['launches'], 1):.1f} pods/launch")
for w in range(16):
    if d[16 + w]:
        extra = f"  wait {d[6 + w] / pods:8.0f}" if w < 3 else ""
        print(f"  wave {w:2d} work {d[16 + w] / pods:8.0f} cycles/pod{extra}")
it = (d[16] + d[6]) / pods
print(f"  iteration {it:.0f} cycles/pod (wave 0 work + wait) -> stamp clock {it / ns:.2f} GHz")
print(f"  lanes passing the K1 bound {d[9] / pods:.2f}/pod, (wave, k) K1 evaluations {d[10] / pods:.2f}/pod, "
      f"can-win lanes {d[11] / pods:.2f}/pod, zero pod-i+2 bound {d[12] / pods:.2f}/pod (per wave x k)")
