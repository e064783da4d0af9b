"""Dev tool (not a test): statistics of the batched resolve on a C3 prefix, exact integer model.

For each batch of B pods: the snapshot top-L lists, then the sequential walk with the touched set
(expiry nodes pre-inserted + in-batch winners).  Per pod it records how many touched entries exist,
how many of them have an exact key >= the pod's list candidate (the work a resolver cannot prune),
how many pass a pod-specific float bound (prune_tmax), and where the winner came from.

    python tests/dev/resolve_stats.py --nodes 50000 --batches 12
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import encode, tracegen  # noqa: E402


def scores(ac, am, ag, ap, rc, rm, rg, nr, taint, label, p):
    """exact total+1 (0 = not a candidate), fit + taint + selector filters, LR + BA (w 1, 1)"""
    qc, qm, qg = p["req"]
    ok = (nr < ap) & (rc + qc <= ac) & (rm + qm <= am) & (rg + qg <= ag)
    ok &= (taint & ~p["tol"]) == 0
    ok &= (label & p["sel"]) == p["sel"]
    uc, um = rc + qc, rm + qm
    lc = np.where((ac > 0) & (uc <= ac), (ac - uc) * 10 // np.maximum(ac, 1), 0)
    lm = np.where((am > 0) & (um <= am), (am - um) * 10 // np.maximum(am, 1), 0)
    ba_on = (ac > 0) & (am > 0) & (uc < ac) & (um < am)
    # exact BA in int64: C3 quantities are multiples of 100m cpu and 256Mi memory (milli-units)
    mu = (256 << 20) * 1000
    Ac, Am = ac // 100, am // mu
    Uc, Um = uc // 100, um // mu
    Dd = Ac * Am
    X = np.abs(Uc * Am - Um * Ac)
    ba = np.where(ba_on, (10 * (Dd - X)) // np.maximum(Dd, 1), 0)
    tot = (lc + lm) // 2 + ba
    return np.where(ok, tot + 1, 0)


def keys(t1, nodes):
    return np.where(t1 > 0, (t1.astype(np.int64) << 32) | (0xFFFFFFFF - nodes), 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pods", type=int, default=20_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--batches", type=int, default=10)
    ap.add_argument("--skip", type=int, default=8000, help="pods bound sequentially before measuring")
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--overlap", action="store_true",
                    help="lists from the snapshot before the previous batch; its modified nodes touched")
    a = ap.parse_args()
    tr = tracegen.c3_trace(n_nodes=a.nodes, n_pods=a.pods)
    enc = encode.encode_trace(tr)
    al = enc["alloc"]
    ac, am, ag, apd = al[:, 0].copy(), al[:, 1].copy(), al[:, 2].copy(), al[:, 3].copy()
    N = a.nodes
    rc = np.zeros(N, np.int64); rm = np.zeros(N, np.int64); rg = np.zeros(N, np.int64); nr = np.zeros(N, np.int64)
    taint = enc["taint"].astype(np.uint64); label = enc["label"].astype(np.uint64)
    P = enc["pods"]
    req = P["req"].reshape(-1, 3)
    km = P["keymask"]
    req = req * ((km[:, None] >> np.arange(3)) & 1)
    tol = P["tol"].astype(np.uint64); sel = P["sel"].astype(np.uint64)
    poff, psec = P["phase_off"], P["phase_sec"]
    S = np.add.reduceat(psec.astype(np.int64), poff[:-1]) if len(psec) else np.zeros(len(req))
    dur = -(-S // tr["tick_seconds"])
    nid = np.arange(N, dtype=np.int64)
    fin = {}  # tick -> list of pods
    node_of = np.full(len(req), -1)

    def pod(j):
        return dict(req=req[j], tol=tol[j], sel=sel[j])

    def expire(t):
        out = []
        for q in fin.pop(t, []):
            n = node_of[q]
            rc[n] -= req[q, 0]; rm[n] -= req[q, 1]; rg[n] -= req[q, 2]; nr[n] -= 1
            out.append(n)
        return out

    def bind(j, n, t):
        qc, qm, qg = req[j]
        ok = (nr[n] < apd[n]) and rc[n] + qc <= ac[n] and rm[n] + qm <= am[n] and rg[n] + qg <= ag[n]
        node_of[j] = n
        if ok and dur[j] > 0:
            rc[n] += qc; rm[n] += qm; rg[n] += qg; nr[n] += 1
            fin.setdefault(t + dur[j], []).append(j)

    st = dict(T=[], ge=[], win_list=0, win_touched_batch=0, win_touched_exp=0, exhausted=0, pods=0,
              lk_rank=[], pre=[], Tact=[], bnd=[], grp=[], grp_pass=[], grp_act=[], grp_act_pass=[])

    def tbound(n_idx, p):
        """prune_tmax's float upper bound of total (ks_device.h), vectorised, filters ignored"""
        qc, qm, _ = p["req"]
        a_c, a_m = ac[n_idx].astype(np.float32), am[n_idx].astype(np.float32)
        ic = np.where(a_c > 0, 1 / np.maximum(a_c, 1), 0).astype(np.float32)
        im = np.where(a_m > 0, 1 / np.maximum(a_m, 1), 0).astype(np.float32)
        fc = np.where(a_c > 0, (a_c - rc[n_idx]) * ic, -1) - qc * ic
        fm = np.where(a_m > 0, (a_m - rm[n_idx]) * im, -1) - qm * im
        lc = np.where(fc > -1.5e-5, np.floor(10 * fc + 1.5e-5), 0)
        lm = np.where(fm > -1.5e-5, np.floor(10 * fm + 1.5e-5), 0)
        tot = (lc + lm) // 2
        tot = tot + np.where((fc > -1.5e-5) & (fm > -1.5e-5), np.floor(10 - 10 * np.abs(fc - fm) + 3e-5), 0)
        return tot.astype(np.int64)
    j = 0
    # warm-up: sequential
    while j < a.skip:
        t = j + 1
        expire(t)
        k = scores(ac, am, ag, apd, rc, rm, rg, nr, taint, label, pod(j))
        bind(j, int(np.argmax(keys(k, nid))), t)
        j += 1
    snap = (rc.copy(), rm.copy(), rg.copy(), nr.copy())
    prev_mod = set()
    for b in range(a.batches):
        s = j
        t = s + 1
        head = set(int(node_of[q]) for q in fin.get(t, []))
        expire(t)
        # snapshot lists (overlap: the state before the previous batch, as a scan running beside
        # the previous resolve would see it)
        src = snap if a.overlap else (rc, rm, rg, nr)
        snap = (rc.copy(), rm.copy(), rg.copy(), nr.copy())
        lists = []
        for i in range(a.batch):
            k = keys(scores(ac, am, ag, apd, src[0], src[1], src[2], src[3], taint, label, pod(s + i)), nid)
            top = np.argsort(-k)[:a.L]
            lists.append([(int(k[x]), int(x)) for x in top if k[x] > 0])
        # pre-inserted expiry nodes of the window
        pre = set()
        for i in range(1, a.batch):
            for q in fin.get(s + i + 1, []):
                pre.add(int(node_of[q]))
        if a.overlap:
            pre |= prev_mod | head
        st["pre"].append(len(pre))
        touched = set(pre)
        modified = set()
        order = list(pre)  # entry numbering: pre-inserted, then in-batch winners
        act_order = []     # entry numbering by activation (first bind or expiry in the batch)
        for i in range(a.batch):
            jj = s + i
            tt = jj + 1
            if i > 0:
                for n_ in expire(tt):
                    if n_ not in modified:
                        modified.add(n_)
                        act_order.append(n_)
            k = keys(scores(ac, am, ag, apd, rc, rm, rg, nr, taint, label, pod(jj)), nid)
            lst = lists[i]
            unt = [(kk, x) for kk, x in lst if x not in touched]
            if not unt and len(lst) == a.L:
                st["exhausted"] += 1
                j = jj
                break
            lk = unt[0][0] if unt else 0
            if unt:
                st["lk_rank"].append(lst.index(unt[0]))
            T = np.fromiter(touched, np.int64) if touched else np.zeros(0, np.int64)
            st["T"].append(len(T))
            st["ge"].append(int((k[T] >= lk).sum()) if len(T) else 0)
            st["Tact"].append(len(modified))
            if len(order):
                E = np.array(order, np.int64)
                bk = keys(tbound(E, pod(jj)) + 1, E)
                ok_ = bk >= lk
                st["bnd"].append(int(ok_.sum()))
                g = np.arange(len(E)) // 64
                st["grp"].append(int(g.max()) + 1)
                st["grp_pass"].append(len(set(g[ok_])))
            if act_order:
                E = np.array(act_order, np.int64)
                bk = keys(tbound(E, pod(jj)) + 1, E)
                ok_ = bk >= lk
                g = np.arange(len(E)) // 64
                st["grp_act"].append(int(g.max()) + 1)
                st["grp_act_pass"].append(len(set(g[ok_])))
            w = int(np.argmax(k))
            if w in touched:
                if w in pre:
                    st["win_touched_exp"] += 1
                else:
                    st["win_touched_batch"] += 1
            else:
                st["win_list"] += 1
                assert k[w] == lk, (k[w], lk)
            if w not in touched:
                order.append(w)
            if w not in modified:
                modified.add(w)
                act_order.append(w)
            touched.add(w)
            bind(jj, w, tt)
            st["pods"] += 1
            j = jj + 1
        prev_mod = set(modified) | head
    T = np.array(st["T"]); ge = np.array(st["ge"])
    print(f"pods {st['pods']}  exhausted stops {st['exhausted']}  pre-inserted/batch {np.mean(st['pre']):.0f}")
    print(f"touched T: mean {T.mean():.0f} max {T.max()}")
    print(f"touched entries with exact key >= list cand: mean {ge.mean():.2f}  p90 {np.percentile(ge, 90):.0f}  max {ge.max()}")
    print(f"winner: list {st['win_list']}  touched(batch) {st['win_touched_batch']}  touched(expiry) {st['win_touched_exp']}")
    print(f"list cand rank histogram: {np.bincount(st['lk_rank'])}")
    print(f"modified (active) entries: mean {np.mean(st['Tact']):.0f}  max {np.max(st['Tact'])}")
    print(f"entries passing the float bound: mean {np.mean(st['bnd']):.2f}  p90 {np.percentile(st['bnd'], 90):.0f}")
    print(f"64-entry groups: mean {np.mean(st['grp']):.2f}, with a bound pass {np.mean(st['grp_pass']):.2f}")
    print(f"activation-ordered groups: mean {np.mean(st['grp_act']):.2f}, with a bound pass {np.mean(st['grp_act_pass']):.2f}")


if __name__ == "__main__":
    main()
