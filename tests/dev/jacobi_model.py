"""Dev tool (not a test): how many parallel (Jacobi) sweeps does a batch of the resolve need?

Exact integer model on a C3 prefix.  For a batch of B pods with the state S before it:
  * truth: the sequential loop (pod i binds the argmax over every node of its key on the state
    after pods < i, expiries applied at their ticks);
  * Jacobi: w^0_i = argmax ignoring the batch's own binds; sweep t+1 recomputes every pod's
    argmax on the state that the binds w^t_{<i} (with their admission) and the expiries give.
    After sweep t the first t pods are exact (induction), so the fixed point is the sequential
    result; the question is how many sweeps a batch needs in practice.

    python tests/dev/jacobi_model.py --batches 6 --batch 256
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from resolve_stats import keys, scores  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import encode, tracegen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pods", type=int, default=20_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--skip", type=int, default=8000)
    ap.add_argument("--K", type=int, default=48, help="baseline list length per pod")
    a = ap.parse_args()
    tr = tracegen.c3_trace(n_nodes=a.nodes, n_pods=a.pods)
    enc = encode.encode_trace(tr)
    al = enc["alloc"]
    ac, am, ag, apd = (al[:, k].copy() for k in range(4))
    N = a.nodes
    st = np.zeros((4, N), np.int64)  # rc rm rg nr
    taint = enc["taint"].astype(np.uint64)
    label = enc["label"].astype(np.uint64)
    P = enc["pods"]
    km = P["keymask"]
    req = P["req"].reshape(-1, 3) * ((km[:, None] >> np.arange(3)) & 1)
    tol = P["tol"].astype(np.uint64)
    sel = P["sel"].astype(np.uint64)
    S = np.add.reduceat(P["phase_sec"].astype(np.int64), P["phase_off"][:-1])
    S = np.where(np.diff(P["phase_off"]) > 0, S, 0)
    dur = np.where(S > 0, -(-S // tr["tick_seconds"]), 0)
    nid = np.arange(N, dtype=np.int64)
    node_of = np.full(len(req), -1)
    ok_of = np.zeros(len(req), bool)

    def pod(j):
        return dict(req=req[j], tol=tol[j], sel=sel[j])

    def key_on(j, n, s):  # exact key of pod j on nodes n with state columns s (4 x len(n))
        k = scores(ac[n], am[n], ag[n], apd[n], s[0], s[1], s[2], s[3], taint[n], label[n], pod(j))
        return keys(k, n)

    def fits(j, n, s):
        q = req[j]
        return bool(s[3] < apd[n] and s[0] + q[0] <= ac[n] and s[1] + q[1] <= am[n] and s[2] + q[2] <= ag[n])

    # expiry ticks of bound pods: tick -> pods
    fin = {}

    def apply_expiries(t):
        for q in fin.pop(t, []):
            n = node_of[q]
            st[:3, n] -= req[q]
            st[3, n] -= 1

    def bind_seq(j, n, t):
        ok = fits(j, n, st[:, n])
        node_of[j] = n
        ok_of[j] = ok
        if ok and dur[j] > 0:
            st[:3, n] += req[j]
            st[3, n] += 1
            fin.setdefault(t + dur[j], []).append(j)

    j = 0
    while j < a.skip:  # warm-up: the exact sequential loop (bulk arrivals: pod j binds at tick j + 1)
        t = j + 1
        apply_expiries(t)
        k = keys(scores(ac, am, ag, apd, st[0], st[1], st[2], st[3], taint, label, pod(j)), nid)
        bind_seq(j, int(np.argmax(k)), t)
        j += 1

    sweeps_needed = []
    for b in range(a.batches):
        s0 = j
        B = a.batch
        t0 = s0 + 1
        apply_expiries(t0)
        snap = st.copy()
        fin_snap = {t: list(v) for t, v in fin.items()}
        # pre-batch expiries inside the batch window: node -> list of (tick, pod)
        exp_in = {}
        for t in range(t0 + 1, t0 + B):
            for q in fin_snap.get(t, []):
                exp_in.setdefault(int(node_of[q]), []).append((t, q))
        # ---- truth: sequential
        truth = []
        for i in range(B):
            jj, tt = s0 + i, s0 + i + 1
            if i > 0:
                apply_expiries(tt)
            k = keys(scores(ac, am, ag, apd, st[0], st[1], st[2], st[3], taint, label, pod(jj)), nid)
            w = int(np.argmax(k))
            truth.append(w)
            bind_seq(jj, w, tt)
        truth = np.array(truth)
        j = s0 + B
        # ---- Jacobi
        # baseline per pod: snapshot keys with the pre-batch expiries of its tick; top-K over
        # nodes with no pre-batch expiry in the window (those are evaluated exactly per pod)
        E = np.array(sorted(exp_in), np.int64)
        isexp = np.zeros(N, bool)
        isexp[E] = True
        base_top = []
        for i in range(B):
            k = keys(scores(ac, am, ag, apd, snap[0], snap[1], snap[2], snap[3], taint, label, pod(s0 + i)), nid)
            k = np.where(isexp, 0, k)
            top = np.argsort(-k)[:a.K]
            base_top.append([(int(k[x]), int(x)) for x in top if k[x] > 0])

        def state_at(i, n, w, okv):
            """state of node n at pod i's bind (tick t0 + i) given binds w[:i] (admission okv)"""
            tt = t0 + i
            s = snap[:, n].copy()
            for tq, q in exp_in.get(n, []):
                if tq <= tt:
                    s[:3] -= req[q]
                    s[3] -= 1
            for jx in range(i):
                if w[jx] == n and okv[jx] and dur[s0 + jx] > 0:
                    if t0 + jx + dur[s0 + jx] > tt:  # still running at tt (expiry applied at its tick)
                        s[:3] += req[s0 + jx]
                        s[3] += 1
            return s

        def sweep(w):
            """one Jacobi sweep: every pod's argmax given the binds w (admission recomputed in order)"""
            okv = np.zeros(B, bool)
            for i in range(B):
                okv[i] = fits(s0 + i, int(w[i]), state_at(i, int(w[i]), w, okv))
            neww = np.zeros(B, np.int64)
            for i in range(B):
                cand = set(int(x) for x in w[:i]) | set(int(x) for x in E)
                best, bn = 0, -1
                for n in cand:
                    kk = int(key_on(s0 + i, np.array([n]), state_at(i, n, w, okv)[:, None])[0])
                    if kk > best:
                        best, bn = kk, n
                # best baseline node not in cand
                for kk, x in base_top[i]:
                    if x not in cand:
                        if kk > best:
                            best, bn = kk, x
                        break
                else:
                    if len(base_top[i]) == a.K:
                        raise RuntimeError("baseline list exhausted; raise --K")
                neww[i] = bn
            return neww

        w = sweep(np.full(B, -1))  # sweep over "no binds": w^0
        t = 0
        while True:
            nw = sweep(w)
            t += 1
            if (nw == w).all():
                break
            w = nw
        assert (w == truth).all(), "Jacobi fixed point differs from the sequential result"
        sweeps_needed.append(t)
        # prefix-exact count per sweep
        print(f"batch {b}: {t} sweeps to the fixed point (= sequential); "
              f"distinct winners {len(set(truth.tolist()))}, expiry-node winners {int(isexp[truth].sum())}", flush=True)
    print("sweeps per batch:", sweeps_needed)


if __name__ == "__main__":
    main()
