"""CRC of the C3 trace's first binds at several batch sizes (must agree), plus the first pod where
two batch sizes disagree.  KS_OVERLAP in the environment selects the overlap."""
import os, sys, zlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import tracegen, encode
from kubesim_amd.engine import Engine
P = int(os.environ.get("PODS", "200000"))
tr = tracegen.c3_trace(n_pods=P)
enc = encode.encode_trace(tr)
res = {}
for B in [int(x) for x in sys.argv[1:]] or [0, 97]:
    eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), batch_pods=B)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    eng.submit(enc["pods"])
    b = eng.step(P)
    res[B] = b
    print(f"batch {B}: {len(b)} binds, crc {zlib.crc32(b['node'].tobytes() + b['status'].tobytes()):08x}", flush=True)
    eng.close()
ks = list(res)
for k in ks[1:]:
    d = np.nonzero(res[ks[0]]["node"] != res[k]["node"])[0]
    print(f"batch {ks[0]} vs {k}: first difference at pod {d[0] if len(d) else None}")
