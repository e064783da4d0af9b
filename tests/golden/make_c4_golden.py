"""Regenerate tests/golden/c4_golden.json: per-scenario golden results of the C4 workload
(BASELINE.json configs[3]: 1024 what-if scenarios x 2,000 nodes x 10,000 pods, tracegen C4
distributions, Filter fit+taint+selector -> LeastRequested + BalancedAllocation) from the C oracle
(oracle/ks_oracle.c, the restatement of kubesim/kubesim.go:90-225 with kubesim/node/node.go:36-60
admission and kubesim/pod/pod.go:47-69 usage).  TEST INFRASTRUCTURE ONLY.

Per scenario: the oracle's return code (0, or the aborting error: NotFound), the number of binds,
blake2b-128 of the binds' (node int32, status int32, tick int64) arrays in pod order, and
blake2b-128 of usage[n][3] (int64) at the end of the run.  tests/test_engine_gpu_config_size.py
compares every scenario of the engine's group run with these.

    python tests/golden/make_c4_golden.py [--procs 8]
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-simulator_amd"), os.path.join(ROOT, "oracle")]

from kubesim_amd import tracegen  # noqa: E402
from pyoracle import COracle  # noqa: E402

S, N, P = 1024, 2000, 10_000
SCORERS = ((1, 1, 0), (2, 1, 0))
OUT = os.path.join(HERE, "c4_golden.json")


def digest(*arrays):
    h = hashlib.blake2b(digest_size=16)
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def one(s):
    tr = tracegen.c4_scenario(s, n_nodes=N, n_pods=P)
    ora = COracle(tr, filter_mode=1, filters=7, scorers=SCORERS)
    ora.submit(tr)
    b, rc = ora.step(P, cap=P)
    res = [s, int(rc), int(len(b["pod"])),
           digest(np.asarray(b["node"], np.int32), np.asarray(b["status"], np.int32), np.asarray(b["tick"], np.int64)),
           digest(ora.usage().astype(np.int64))]
    ora.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    t0 = time.time()
    with mp.Pool(args.procs) as pool:
        rows = []
        for i, r in enumerate(pool.imap(one, range(S), chunksize=4)):
            rows.append(r)
            if (i + 1) % 64 == 0:
                print(f"{i + 1}/{S} scenarios ({time.time() - t0:.0f} s)", flush=True)
    out = {"generator": "tests/golden/make_c4_golden.py", "scenarios": S, "nodes": N, "pods": P,
           "mode": "feeds_all_lrba", "scorers": [list(x) for x in SCORERS],
           "digest": "blake2b-128 of (node int32, status int32, tick int64) of the binds; usage[n][3] int64 at the end",
           "columns": ["scenario", "rc", "binds", "bind_digest", "usage_digest"],
           "rows": rows, "aborted": sum(1 for r in rows if r[1] != 0),
           "oracle_seconds": round(time.time() - t0, 1)}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
