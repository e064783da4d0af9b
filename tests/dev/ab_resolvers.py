"""A/B of the resolvers on the C3 bench workload (and C5 with --c5): per-launch resolve / scan /
other device time (HIP events), pods per launch, wall pods/s and a CRC of the binds (must agree).
    python tests/dev/ab_resolvers.py [--c5] [--noprof] [one_pod chunk chunk@256 ...]   (@B = batch)
--noprof: no per-kernel events (the overlapped chain runs; only the wall rate and CRC mean anything)"""
import os, sys, time, zlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib
if os.environ.get("KS_DIAG_LIB"):
    _lib.LIB_PATH = lib_path(os.environ["KS_DIAG_LIB"])
from kubesim_amd import tracegen, encode
from kubesim_amd.engine import Engine
args = [x for x in sys.argv[1:] if not x.startswith("--")]
c5 = "--c5" in sys.argv
names = args or ["chunk", "one_pod"]
FLAGS = {"one_pod": 8, "chunk": 64}
tr = tracegen.c5_trace(n_pods=120_000) if c5 else tracegen.c3_trace(n_pods=200_000)
enc = encode.encode_trace(tr)
for rep in range(2):
    for nm in names:
        nm0, _, bp = nm.partition("@")  # name@B: batch of B pods
        base = nm0
        eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), engine_flags=FLAGS[base],
                     batch_pods=int(bp) if bp else 0)
        eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
        eng.submit(enc["pods"])
        eng.step(32768)
        if "--noprof" not in sys.argv:  # (profiling times each kernel: no overlap)
            eng.set_profiling(True)
        t = time.perf_counter(); b = eng.step(65536); dt = time.perf_counter() - t
        st = eng.last_step_stats()
        nl = max(st["launches"], 1)
        crc = zlib.crc32(np.ascontiguousarray(b["node"]).tobytes() + np.ascontiguousarray(b["status"]).tobytes())
        extra = ""
        if os.environ.get("KS_DIAG_LIB"):
            d = eng.debug_counters()
            extra = " diag " + " ".join(str(int(x)) for x in d[5:16])
            nl_ = max(int(d[5]), 1)
            extra += " | cycles/launch: " + " ".join(f"{int(x) // nl_}" for x in d[16:24])
        print(f"{nm:10s}: resolve {st['resolve_ms'] / nl * 1e3:6.1f} us/launch ({st['resolve_ms'] * 1e6 / max(st['pods'], 1):5.0f} ns/pod), "
              f"scan {st['scan_ms'] / nl * 1e3:5.1f}, other {st['other_ms'] / nl * 1e3:5.1f}; {st['pods'] / nl:6.1f} pods/launch; "
              f"{65536 / dt:8.0f} pods/s; crc {crc:08x}{extra}", flush=True)
        eng.close()
