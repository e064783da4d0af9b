"""Digests of tests/golden/full_run.json (made by tests/golden/make_full_run.py from the oracle):
blake2b-128 of a window's binds (node int32, status int32, tick int64, pod order) and of
usage[n][3] (int64) at a tick."""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "full_run.json")


def digest(*arrays):
    h = hashlib.blake2b(digest_size=16)
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def bind_digest(b):
    return digest(np.asarray(b["node"], np.int32), np.asarray(b["status"], np.int32), np.asarray(b["tick"], np.int64))


def load(name):
    with open(GOLDEN) as f:
        return json.load(f).get(name)


def check_engine_run(eng, g, label=""):
    """Step `eng` window by window over the golden run `g`; every window's binds and every sampled
    usage matrix must match.  Returns the binds of the whole run."""
    usage = {int(t): d for t, d in g["usage_digests"]}
    out, done = [], 0
    nwin = len(g["bind_digests"])
    for w in range(nwin):
        k = min(g["window"], g["pods"] - done)
        b = eng.step(k)
        assert len(b) == k, (label, w, len(b), k)
        assert int(b["pod"][0]) == done
        assert bind_digest(b) == g["bind_digests"][w], f"{label}: window {w} (pods {done}..{done + k}) differs"
        done += k
        if eng.tick in usage:
            assert digest(eng.usage().astype(np.int64)) == usage[eng.tick], f"{label}: usage at tick {eng.tick}"
        out.append(b)
    return np.concatenate(out)
