"""Dev tool (not a test): whole-run goldens (tests/golden/full_run.json) at many batch sizes — every
batch size moves the chunk resolver's batch and chunk boundaries, so alignment-dependent paths
(segment overflow, exhausted lists, slot cuts, rescans) are exercised at other pods.
    python tests/dev/batch_sweep.py c5|c3|c3lit B0 B1 [STEP] [FLAGS]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402
_lib.LIB_PATH = lib_path(os.environ.get("KS_LIB", "libks_engine.so"))
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402
import full_run_digest  # noqa: E402

name, b0, b1 = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
step = int(sys.argv[4]) if len(sys.argv) > 4 else 1
flags = int(sys.argv[5]) if len(sys.argv) > 5 else 0
g = full_run_digest.load(name)
if name == "c5":
    tr = tracegen.c5_trace(n_pods=g["pods"])
else:
    tr = tracegen.c3_trace(n_nodes=50_000, n_pods=g["pods"])
enc = encode.encode_trace(tr)
fm = 0 if name == "c3lit" else 1
bad = 0
for B in range(b0, b1, step):
    t0 = time.time()
    e = Engine(tick_seconds=10, filter_mode=fm, filters=7, scorers=((1, 1, 0), (2, 1, 0)), batch_pods=B, engine_flags=flags)
    e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    e.submit(enc["pods"])
    done, first = 0, None
    for w, want in enumerate(g["bind_digests"]):
        k = min(g["window"], g["pods"] - done)
        b = e.step(k)
        if full_run_digest.bind_digest(b) != want and first is None:
            first = w
        done += k
    e.close()
    bad += first is not None
    print(f"batch {B}: {'window ' + str(first) + ' differs' if first is not None else 'ok'} ({time.time() - t0:.1f} s)", flush=True)
print(f"{bad} batch sizes off the golden")
