"""Hand-derived known-answer test for BASELINE.json configs[0] (config/sample.yml +
examples/main.go), written from the reference's rules, not from any implementation:

* pod n is submitted at tick n+1 (examples/main.go:84-85: elapsed/5 >= n, tick 10 s) and
  binds at that tick (one pod per tick, kubesim/kubesim.go:105-121);
* every node scores 1 (examples/main.go:147-155); the tie goes to the lowest index: node-0;
* requests {cpu 3, memory 5Gi, gpu 1} vs node-0 capacity {4, 8Gi, 1, pods 2}
  (config/sample.yml:16-24): a pod is OverCapacity iff the previous pod is still running
  (cpu 3+3 > 4; kubesim/node/node.go:44-47); a pod runs 5 s + 10 s = 15 s, i.e. at its
  bind tick and the next one (kubesim/pod/pod.go:67-69) — so even pods are Ok, odd pods
  OverCapacity;
* usage of node-0 after the bind at tick t: t odd → phase 0 of the pod bound now
  {1, 2Gi, 0}; t even → phase 1 of the pod bound at t-1 {2, 4Gi, 1} (pod.go:47-63).
Quantities in milli-units.
"""
import json, os
GI = 1 << 30
T = 60
binds, usage = [], []
for t in range(1, T + 1):
    n = t - 1
    binds.append([n, 0, t, 0 if n % 2 == 0 else 1])
    node0 = [1000, 2 * GI * 1000, 0] if t % 2 == 1 else [2000, 4 * GI * 1000, 1000]
    usage.append([node0, [0, 0, 0]])
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "c1_kat.json"), "w") as f:
    json.dump(dict(config="C1", ticks=T, binds=binds, usage=usage), f)
