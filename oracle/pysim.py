"""Independent pure-Python restatement of the kubesim scheduling loop.

TEST INFRASTRUCTURE ONLY (see oracle/ks_oracle.h).  Written separately from the C oracle
and on a different representation — resource lists are ``dict[name] -> int`` keyed by the
reference's resource names, taints/tolerations/labels are compared as *strings*, totals are
rebuilt from every pod ever stored on the node (no pruning), and the argmax walks a dict
built in node order — so that agreement between the two is evidence about the semantics,
not a shared bug.  Pure-Python loops: small cases only.

Cites the same reference lines as ks_oracle.c:
kubesim/kubesim.go:90-225, kubesim/node/node.go:36-118, kubesim/node/resource.go:10-61,
kubesim/pod/pod.go:47-69,148-162, vendor/k8s.io/api/core/v1/toleration.go:37-56.
"""
from __future__ import annotations

from fractions import Fraction

RES = ("cpu", "memory", "nvidia.com/gpu")
EFFECTS = {1: "NoSchedule", 2: "PreferNoSchedule", 3: "NoExecute"}
OPS = {0: "Equal", 1: "Exists", 2: "Bogus"}


def _rlist(vals, has):
    return {RES[k]: int(vals[k]) for k in range(3) if (int(has) >> k) & 1}


def resource_list_sum(r1, r2):
    """kubesim/node/resource.go:10-21"""
    out = dict(r1)
    for k, v in r2.items():
        out[k] = out.get(k, 0) + v
    return out


def resource_list_ge(r1, r2):
    """kubesim/node/resource.go:52-61"""
    for k, v in r2.items():
        if k not in r1 or r1[k] < v:
            return False
    return True


class PySim:
    def __init__(self, trace, *, filter_mode=0, filters=0, scorers=((0, 1, 1),)):
        self.s = trace["strings"]
        self.tick_s = trace["tick_seconds"]
        nd = trace["nodes"]
        self.n = nd["n"]
        self.cap = []
        self.taints = []
        self.labels = []
        for i in range(self.n):
            c = _rlist(nd["alloc"][i][:3], nd["alloc_has"][i])
            if int(nd["alloc_has"][i]) & 8:
                c["pods"] = int(nd["alloc"][i][3])
            self.cap.append(c)
            self.taints.append([(self.s[k], self.s[v], EFFECTS[int(e)])
                                for k, v, e in nd["taint"][nd["taint_off"][i]:nd["taint_off"][i + 1]]])
            self.labels.append({self.s[k]: self.s[v]
                                for k, v in nd["label"][nd["label_off"][i]:nd["label_off"][i + 1]]})
        self.filter_mode = filter_mode
        self.filters = filters
        self.scorers = list(scorers)
        self.pods = []
        self.node_pods = [dict() for _ in range(self.n)]  # key -> pod index (sync.Map)
        self.tick = 0
        self.qhead = 0
        self.err = None

    def submit(self, trace):
        p = trace["pods"]
        for j in range(p["m"]):
            spec = []
            for f in range(p["phase_off"][j], p["phase_off"][j + 1]):
                spec.append((int(p["phase_sec"][f]), _rlist(p["phase_use"][f], p["phase_has"][f])))
            tols = []
            for t in p["tol"][p["tol_off"][j]:p["tol_off"][j + 1]]:
                k, op, v, e = (int(x) for x in t)
                tols.append(dict(key=self.s[k], op=OPS[op], value=self.s[v],
                                 effect="" if e == 0 else EFFECTS[e]))
            sel = {self.s[k]: self.s[v] for k, v in p["sel"][p["sel_off"][j]:p["sel_off"][j + 1]]}
            self.pods.append(dict(arrival=int(p["arrival"][j]), req=_rlist(p["req"][j], p["req_has"][j]),
                                  tols=tols, sel=sel, spec=spec, key=int(p["key_id"][j]),
                                  flags=int(p["flags"][j]), node=None, status=None, t0=None))

    # -- pod.go ------------------------------------------------------------------------------
    def _passed(self, pod, t):
        if pod["status"] != "Ok":
            return 0
        x = (t - pod["t0"]) * self.tick_s
        x &= 0xFFFFFFFF
        return x - (1 << 32) if x >= (1 << 31) else x

    @staticmethod
    def _i32(x):
        x &= 0xFFFFFFFF
        return x - (1 << 32) if x >= (1 << 31) else x

    def _total_seconds(self, pod):
        acc = 0
        for sec, _ in pod["spec"]:
            acc = self._i32(acc + sec)
        return acc

    def _running(self, pod, t):
        return pod["status"] == "Ok" and self._passed(pod, t) < self._total_seconds(pod)

    def _usage(self, pod, t):
        if not self._running(pod, t):
            return {}
        passed = self._passed(pod, t)
        acc = 0
        for sec, use in pod["spec"]:
            acc = self._i32(acc + sec)
            if passed < acc:
                return use
        return {}

    # -- node.go -----------------------------------------------------------------------------
    def _total_request(self, n, t):
        total = {}
        for j in self.node_pods[n].values():
            if self._running(self.pods[j], t):
                total = resource_list_sum(total, self.pods[j]["req"])
        return total

    def _running_num(self, n, t):
        return sum(1 for j in self.node_pods[n].values() if self._running(self.pods[j], t))

    def _fits(self, n, pod, t):
        new_total = resource_list_sum(self._total_request(n, t), pod["req"])
        pods_cap = self.cap[n].get("pods", 0)
        return resource_list_ge(self.cap[n], new_total) and not (self._running_num(n, t) >= pods_cap)

    # -- build-defined plugins ----------------------------------------
    @staticmethod
    def _tolerates(tol, taint):
        key, value, effect = taint
        if tol["effect"] and tol["effect"] != effect:
            return False
        if tol["key"] and tol["key"] != key:
            return False
        if tol["op"] == "Equal":
            return tol["value"] == value
        return tol["op"] == "Exists"

    def _taint_ok(self, n, pod):
        for taint in self.taints[n]:
            if taint[2] == "PreferNoSchedule":
                continue
            if not any(self._tolerates(tl, taint) for tl in pod["tols"]):
                return False
        return True

    def _selector_ok(self, n, pod):
        return all(self.labels[n].get(k) == v for k, v in pod["sel"].items())

    def _used(self, n, pod, t, name):
        return self._total_request(n, t).get(name, 0) + pod["req"].get(name, 0)

    def _lr(self, n, pod, t):
        s = 0
        for name in ("cpu", "memory"):
            a, u = self.cap[n].get(name, 0), self._used(n, pod, t, name)
            if a <= 0 or u > a:
                continue
            s += (a - u) * 10 // a
        return s // 2

    def _ba(self, n, pod, t):
        ac, am = self.cap[n].get("cpu", 0), self.cap[n].get("memory", 0)
        uc, um = self._used(n, pod, t, "cpu"), self._used(n, pod, t, "memory")
        if ac <= 0 or am <= 0 or uc >= ac or um >= am:
            return 0
        diff = abs(Fraction(uc, ac) - Fraction(um, am))
        return int((1 - diff) * 10)  # exact: floor of a non-negative rational

    def _score_map(self, pod, t):
        nodes = list(range(self.n))
        for bit, fn in ((1, lambda n: self._fits(n, pod, t)), (2, lambda n: self._taint_ok(n, pod)),
                        (4, lambda n: self._selector_ok(n, pod))):
            if self.filters & bit:
                nodes = [n for n in nodes if fn(n)]
        if self.filter_mode == 0:
            nodes = list(range(self.n))
        scores = {}
        for kind, weight, value in self.scorers:
            for n in nodes:
                sc = value if kind == 0 else (self._lr(n, pod, t) if kind == 1 else self._ba(n, pod, t))
                scores[n] = scores.get(n, 0) + sc * weight
        return scores

    def step(self, ticks):
        binds = []
        if self.err:
            return binds, self.err
        for _ in range(ticks):
            t = self.tick + 1
            self.tick = t
            if self.qhead < len(self.pods) and self.pods[self.qhead]["arrival"] <= t:
                j = self.qhead
                self.qhead += 1
                pod = self.pods[j]
                scores = self._score_map(pod, t)
                best, bn = -1, None
                for n in sorted(scores):
                    if scores[n] > best:
                        best, bn = scores[n], n
                if bn is None:
                    self.err = "NotFound"
                    return binds, self.err
                if pod["flags"] & 1:
                    self.err = "InvalidArgument"
                    return binds, self.err
                status = "Ok" if self._fits(bn, pod, t) else "OverCapacity"
                if pod["flags"] & 2:
                    self.err = "InvalidArgument"
                    return binds, self.err
                pod.update(node=bn, status=status, t0=t)
                self.node_pods[bn][pod["key"]] = j
                binds.append((j, bn, t, 0 if status == "Ok" else 1))
        return binds, None

    def usage(self):
        out = []
        for n in range(self.n):
            u = {}
            for j in self.node_pods[n].values():
                u = resource_list_sum(u, self._usage(self.pods[j], self.tick))
            out.append([u.get(r, 0) for r in RES])
        return out
