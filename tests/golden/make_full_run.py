"""Regenerate tests/golden/full_run.json: whole-run golden digests of the C3 and C5 traces from
the C oracle (oracle/ks_oracle.c, the restatement of kubesim/kubesim.go:90-225 with
kubesim/node/node.go:36-60 admission and kubesim/pod/pod.go:47-69 usage), run on this
container's cores with OpenMP over nodes (results identical to the serial oracle:
tests/test_oracle.py::test_threaded_oracle_matches_serial).  TEST INFRASTRUCTURE ONLY.

Every bulk-arrival pod j binds at tick j + 1, so a window of W ticks is a window of W pods.
Per window: blake2b-128 of the binds' (node int32, status int32, tick int64) arrays in pod
order; at sampled window ends: blake2b-128 of usage[n][3] (int64, C order) at that tick.
The GPU test (tests/test_engine_gpu_full_run.py) recomputes the same digests from the engine.

    python tests/golden/make_full_run.py [--threads 8] [--only c3|c5|c3q]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-simulator_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]

from kubesim_amd import tracegen  # noqa: E402
from pyoracle import COracle  # noqa: E402

SCORERS = ((1, 1, 0), (2, 1, 0))  # LeastRequested w1 + BalancedAllocation w1 (the bench's)
OUT = os.path.join(HERE, "full_run.json")

# name -> (trace factory, pods, window, usage-sample every k windows)
RUNS = {
    # bench.py's C3 workload: every pod its default run binds (22 timed + warm-up steps of
    # 32,768 pods and the profiled step stay inside the 1M-pod trace)
    "c3": (lambda: tracegen.c3_trace(n_nodes=50_000, n_pods=1_000_000), 1_000_000, 32_768, 2),
    # bench.py's C5 leg: warm-up + 4 timed + 1 profiled steps of 32,768 pods = 196,608 pods
    "c5": (lambda: tracegen.c5_trace(n_pods=196_608), 196_608, 16_384, 2),
    # C3 with decimal-SI memory requests on binary-SI capacities (the wide evaluator class):
    # the first 131,072 pods of the 1M-pod trace bench.py's c3q leg uses
    "c3q": (lambda: tracegen.slice_pods(tracegen.c3q_trace(n_nodes=50_000, n_pods=1_000_000), 0, 131_072),
            131_072, 16_384, 2),
    # the reference-literal filter mode (kubesim/kubesim.go:182: the Filter result is discarded)
    # on the whole C3 trace: bench.py's c3_literal leg
    "c3lit": (lambda: tracegen.c3_trace(n_nodes=50_000, n_pods=1_000_000), 1_000_000, 32_768, 2),
}
# name -> (filter_mode, mode name in tests/harness.py MODES); default feeds mode
FILTER = {"c3lit": (0, "literal_lrba_filters_ignored")}


def digest(*arrays):
    h = hashlib.blake2b(digest_size=16)
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def bind_digest(node, status, tick):
    return digest(np.asarray(node, np.int32), np.asarray(status, np.int32), np.asarray(tick, np.int64))


def run(name, threads):
    make, pods, window, every = RUNS[name]
    t0 = time.time()
    tr = make()
    assert tr["pods"]["m"] == pods
    fm, mode = FILTER.get(name, (1, "feeds_all_lrba"))
    ora = COracle(tr, filter_mode=fm, filters=7, scorers=SCORERS)
    ora.set_threads(threads)
    ora.submit(tr)
    wins, usage = [], []
    nwin = (pods + window - 1) // window
    for w in range(nwin):
        k = min(window, pods - w * window)
        b, rc = ora.step(k, cap=k)
        assert rc == 0, (name, w, rc, ora.last_error())
        assert len(b["pod"]) == k and int(b["pod"][0]) == w * window
        wins.append(bind_digest(b["node"], b["status"], b["tick"]))
        if (w + 1) % every == 0 or w == nwin - 1:
            usage.append([int(ora.tick), digest(ora.usage().astype(np.int64))])
        print(f"{name}: window {w + 1}/{nwin} ({time.time() - t0:.0f} s)", flush=True)
    return dict(pods=pods, window=window, nodes=tr["nodes"]["n"], mode=mode,
                scorers=[list(s) for s in SCORERS], bind_digests=wins, usage_digests=usage,
                oracle_seconds=round(time.time() - t0, 1), threads=threads)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--only", choices=sorted(RUNS))
    args = ap.parse_args()
    out = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            out = json.load(f)
    out["generator"] = "tests/golden/make_full_run.py"
    out["digest"] = "blake2b-128 of (node int32, status int32, tick int64) per window; usage[n][3] int64"
    for name in ([args.only] if args.only else sorted(RUNS)):
        out[name] = run(name, args.threads)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
