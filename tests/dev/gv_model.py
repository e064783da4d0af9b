"""Dev tool (not a test): design model for an in-LDS sweep resolver (exact integer model, C3).

Per batch of B pods on the snapshot S (state after the previous batch, pod 0's expiries applied):
  * E   = nodes that a pre-batch pod's expiry inside the batch window lands on;
  * cl_i = pod i's static candidates, sorted: its top-L snapshot list entries not in E (snapshot
          key) and the E nodes whose exact key at pod i's tick (expiries due by then) reaches
          thr_i (the list's last key when the list is full, else 1);
  * S_i(W) = the first cl_i entry not in W, D_i(w) = max over the nodes n in W_{<i} of pod i's key
          on n's replayed state (binds with admission, expiries), f_i(w) = max(S_i, D_i).
Chunked sweeps: the batch is cut into chunks of C pods; within a chunk, w^{t+1} = f(w^t) until the
chunk's winners repeat (pods before the chunk are final).  Counts per batch: sweeps, and the
(pod, node) pairs of D that a sweep evaluates (only pods after the previous sweep's first change;
nodes bound before the chunk contribute once per chunk, "cached").

    python tests/dev/gv_model.py --batches 4 --chunks 256,64,32
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
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--skip", type=int, default=8000)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--chunks", default="256,64,32")
    ap.add_argument("--guess", default="none", help="none | excl | dx (chunk seeds, as the kernel's guess)")
    ap.add_argument("--T", type=int, default=3, help="dx: taken entries evaluated per pod")
    a = ap.parse_args()
    tr = tracegen.c3_trace(n_nodes=a.nodes, n_pods=a.pods)
    enc = encode.encode_trace(tr)
    al = enc["alloc"]
    ac, am, ag, apd = (al[:, k].copy() for k in range(4))
    N = a.nodes
    st = np.zeros((4, N), np.int64)
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
    chunks = [int(x) for x in a.chunks.split(",")]

    def pod(j):
        return dict(req=req[j], tol=tol[j], sel=sel[j])

    def key1(j, n, s):
        k = scores(ac[n:n + 1], am[n:n + 1], ag[n:n + 1], apd[n:n + 1], s[0:1], s[1:2], s[2:3], s[3:4],
                   taint[n:n + 1], label[n:n + 1], pod(j))
        return int(keys(k, np.array([n]))[0])

    def fits(j, n, s):
        q = req[j]
        return bool(s[3] < apd[n] and s[0] + q[0] <= ac[n] and s[1] + q[1] <= am[n] and s[2] + q[2] <= ag[n])

    fin = {}

    def apply_expiries(t):
        for q in fin.pop(t, []):
            n = node_of[q]
            st[:3, n] -= req[q]
            st[3, n] -= 1

    def bind_seq(j, n, t):
        ok = fits(j, n, st[:, n])
        node_of[j] = n
        if ok and dur[j] > 0:
            st[:3, n] += req[j]
            st[3, n] += 1
            fin.setdefault(t + dur[j], []).append(j)

    j = 0
    while j < a.skip:
        t = j + 1
        apply_expiries(t)
        k = keys(scores(ac, am, ag, apd, st[0], st[1], st[2], st[3], taint, label, pod(j)), nid)
        bind_seq(j, int(np.argmax(k)), t)
        j += 1

    res = {C: dict(sweeps=[], pairs=[]) for C in chunks}
    clen, rebinds, dwins = [], [], []
    for b in range(a.batches):
        s0, B = j, a.batch
        t0 = s0 + 1
        apply_expiries(t0)
        snap = st.copy()
        fin_snap = {t: list(v) for t, v in fin.items()}
        exp_in = {}
        for t in range(t0 + 1, t0 + B):
            for q in fin_snap.get(t, []):
                exp_in.setdefault(int(node_of[q]), []).append((t, q))
        E = sorted(exp_in)
        isE = np.zeros(N, bool)
        isE[E] = True
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
        rebinds.append(sum(1 for i in range(B) if truth[i] in set(truth[:i].tolist())))

        def e_state(n, i):
            s = snap[:, n].copy()
            for tq, q in exp_in.get(n, []):
                if tq <= t0 + i:
                    s[:3] -= req[q]
                    s[3] -= 1
            return s

        cl = []
        for i in range(B):
            k = keys(scores(ac, am, ag, apd, snap[0], snap[1], snap[2], snap[3], taint, label, pod(s0 + i)), nid)
            top = np.argsort(-k)[:a.L]
            lst = [(int(k[x]), int(x)) for x in top if k[x] > 0]
            thr = lst[-1][0] if len(lst) == a.L else 1
            c = [(kk, x) for kk, x in lst if not isE[x]]
            for n in E:
                kk = key1(s0 + i, n, e_state(n, i))
                if kk >= thr:
                    c.append((kk, n))
            c.sort(reverse=True)
            clen.append(len(c))
            cl.append(c)

        dn = set(x for c in cl for _, x in c)
        print(f"distinct cl nodes {len(dn)}, cl entries {sum(len(c) for c in cl)}, distinct winners {len(set(truth.tolist()))}", flush=True)

        def states(w):
            out = {}
            for n in set(int(x) for x in w if x >= 0):
                s = snap[:, n].copy()
                run = []
                ev = sorted(exp_in.get(n, []))
                col = []
                for i in range(B):
                    tt = t0 + i
                    while ev and ev[0][0] <= tt:
                        _, q = ev.pop(0)
                        s[:3] -= req[q]
                        s[3] -= 1
                    keep = []
                    for te, q in run:
                        if te <= tt:
                            s[:3] -= req[q]
                            s[3] -= 1
                        else:
                            keep.append((te, q))
                    run = keep
                    col.append(s.copy())
                    if w[i] == n and fits(s0 + i, n, s) and dur[s0 + i] > 0:
                        s[:3] += req[s0 + i]
                        s[3] += 1
                        run.append((tt + dur[s0 + i], s0 + i))
                out[n] = col
            return out

        def f_at(w, i, first, stt):
            sv = 0
            for kk, x in cl[i]:
                if not (x in first and first[x] < i):
                    sv = kk
                    break
            dv = 0
            for n, fi in first.items():
                if fi < i:
                    dv = max(dv, key1(s0 + i, n, stt[n][i]))
            v = max(sv, dv)
            return ((0xFFFFFFFF - (v & 0xFFFFFFFF)) if v else -1), dv > sv

        nd = sum(1 for i in range(B) if f_at(truth, i, {int(x): int(np.nonzero(truth == x)[0][0]) for x in truth}, states(truth))[1])
        dwins.append(nd)
        def guess(w, c0, c1):
            """the kernel's chunk guess: exclusion rounds (+ pre-chunk D; dx: + in-chunk D, approx)"""
            pre = set(int(x) for x in w[:c0] if x >= 0)
            wp = w.copy()
            wp[c0:] = -1
            stp = states(wp)
            cd = []
            for i in range(c0, c1):
                ks = sorted(((key1(s0 + i, n, stp[n][i]), n) for n in pre), reverse=True)[:2]
                cd.append([(k, n) for k, n in ks if k > 0])
            al = [[(k, x) for k, x in cl[i] if x not in pre] for i in range(c0, c1)]
            base = {}

            def approx(i, n, binders):
                s = (stp[n][i] if n in stp else e_state(n, i)).copy()  # expiries by pod i's tick
                for j in binders:
                    s[:3] += req[s0 + j]
                    s[3] += 1
                return key1(s0 + i, n, s)

            C = c1 - c0
            cur = [-1] * C
            lo = 0
            while True:
                nwv = list(cur)
                for li in range(lo, C):
                    i = c0 + li
                    taken = {}
                    for lj in range(li):
                        if cur[lj] >= 0:
                            taken.setdefault(cur[lj], []).append(c0 + lj)
                    sk, nw = 0, -1
                    cands = []
                    for k, x in al[li]:
                        if x not in taken:
                            sk, nw = k, x
                            break
                        cands.append(x)
                    best = sk
                    d = [(k, n) for k, n in cd[li] if n not in taken]
                    if d and d[0][0] > best:
                        best, nw = d[0]
                    if a.guess == "dx":
                        ex = cands[:a.T]
                        if cd[li] and cd[li][0][1] in taken:
                            ex.append(cd[li][0][1])
                        for x in ex:
                            k = approx(i, x, taken[x])
                            if k > best:
                                best, nw = k, x
                    nwv[li] = nw
                ch = [li for li in range(C) if nwv[li] != cur[li]]
                cur = nwv
                if not ch:
                    break
                lo = ch[0] + 1
            return np.array(cur)

        sweeps_g = []
        for C in chunks:
            w = np.full(B, -1)
            sweeps = pairs = 0
            for c0 in range(0, B, C):
                c1 = min(B, c0 + C)
                # cached contribution of nodes bound before the chunk: one pass per chunk
                pairs += (c1 - c0) * len(set(w[:c0].tolist()))
                lo = c0  # pods >= lo are recomputed
                if a.guess != "none":
                    w[c0:c1] = guess(w, c0, c1)
                    if os.environ.get("GV_DEBUG"):
                        pre = set(int(x) for x in truth[:c0])
                        for i in range(c0, c1):
                            if w[i] != truth[i]:
                                tn = int(truth[i])
                                print(f"  miss pod {i}: guess {w[i]} truth {tn} pre {tn in pre} "
                                      f"in-chunk-before {tn in set(truth[c0:i].tolist())} in cl {tn in [x for _, x in cl[i]]} "
                                      f"cl rank {[x for _, x in cl[i]].index(tn) if tn in [x for _, x in cl[i]] else -1}")
                                stt_t = states(truth)
                                print(f"    true key {key1(s0+i, tn, stt_t[tn][i]) >> 32} snap key {key1(s0+i, tn, snap[:, tn]) >> 32} "
                                      f"guess-node true key {key1(s0+i, int(w[i]), stt_t[int(w[i])][i]) >> 32 if int(w[i]) in stt_t else key1(s0+i, int(w[i]), e_state(int(w[i]), i)) >> 32} "
                                      f"binders {[j for j in range(c0, i) if truth[j] == tn]} guess binders {[j for j in range(c0, i) if w[j] == tn]} "
                                      f"cl {[(k >> 32, x) for k, x in cl[i][:6]]}")
                                break
                    sweeps_g.append(0)
                while True:
                    first = {}
                    for i, x in enumerate(w[:c1]):
                        if x >= 0 and x not in first:
                            first[int(x)] = i
                    stt = states(w)
                    nw = w.copy()
                    for i in range(lo, c1):
                        nw[i] = f_at(w, i, first, stt)[0]
                        pairs += sum(1 for n, fi in first.items() if c0 <= fi < i)
                    sweeps += 1
                    if a.guess != "none":
                        sweeps_g[-1] += 1
                    ch = np.nonzero(nw[c0:c1] != w[c0:c1])[0]
                    w = nw
                    if len(ch) == 0:
                        break
                    lo = c0 + int(ch[0]) + 1
            assert (w == truth).all(), "fixed point differs from the sequential result"
            res[C]["sweeps"].append(sweeps)
            res[C]["pairs"].append(pairs)
            res[C].setdefault("per_chunk", []).extend(sweeps_g)
            sweeps_g.clear()
        print(f"batch {b}: E {len(E)}, rebinds {rebinds[-1]}, D wins {dwins[-1]}, " +
              ", ".join(f"C={C}: {res[C]['sweeps'][-1]} sweeps {res[C]['pairs'][-1]} pairs" for C in chunks), flush=True)
    cl = np.array(clen)
    print(f"cl length mean {cl.mean():.1f} p99 {np.percentile(cl, 99):.0f} max {cl.max()}; rebinds/batch {np.mean(rebinds):.1f}; D wins/batch {np.mean(dwins):.1f}")
    for C in chunks:
        pc = res[C].get("per_chunk", [])
        print(f"C={C}: sweeps/batch {np.mean(res[C]['sweeps']):.1f}, D pairs/batch {np.mean(res[C]['pairs']):.0f}" +
              (f", full sweeps per chunk {np.mean(pc):.2f} (hist {np.bincount(pc).tolist()})" if pc else ""))


if __name__ == "__main__":
    main()
