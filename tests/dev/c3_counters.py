"""Dev tool (not a test): the C3 bench workload's per-step debug counters on the default engine —
early stops, conditional rescans, list reuses (ks_debug_counters [4], [5], [6]).

    python tests/dev/c3_counters.py [STEPS]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
tr = tracegen.c3_trace()
enc = encode.encode_trace(tr)
e = Engine(tick_seconds=tr["tick_seconds"], filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)))
e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
e.submit(enc["pods"])
prev = [0] * 8
for s in range(steps):
    e.step(32768)
    c = [int(x) for x in e.debug_counters()[:8]]
    d = [c[k] - prev[k] for k in range(8)]
    prev = c
    print(f"step {s}: early stops {d[4]}, rescans {d[5]}, list reuses {d[6]}", flush=True)
