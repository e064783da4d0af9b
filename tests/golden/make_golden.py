"""Regenerate tests/golden/small_traces.json: expected binds + per-tick usage digests of the
seeded cases in tests/golden_traces.py, from the C oracle, each cross-checked bind-for-bind
and usage-for-usage against the independent Python restatement (oracle/pysim.py)."""
import json, os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-simulator_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from golden_traces import CASES, build_trace, run_oracle, usage_digest
from harness import MODES
from pysim import PySim

out = []
for case in CASES:
    res = run_oracle(case)
    fm, fl, sc = MODES[case["mode"]]
    tr = build_trace(case)
    ps = PySim(tr, filter_mode=fm, filters=fl, scorers=sc); ps.submit(tr)
    binds, usage = [], []
    for _ in range(case["ticks"]):
        b, err = ps.step(1)
        binds += [list(x) for x in b]
        if err:
            break
        usage.append(usage_digest(np.array(ps.usage(), dtype=np.int64).reshape(-1, 3)))
    assert binds == res["binds"] and usage == res["usage"], case["name"]
    out.append(dict(name=case["name"], **res))
    print(case["name"], len(res["binds"]), "binds, rc", res["rc"])
with open(os.path.join(HERE, "small_traces.json"), "w") as f:
    json.dump(dict(generator="tests/golden/make_golden.py", cases=out), f)
