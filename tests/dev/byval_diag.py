"""Dev tool (not a test): VERDICT r5 item 1 — the C5 leg on thread-ranks (ks_shard_host), window by
window against the committed oracle digests, with every rank's binds saved and compared with each
other, so a diagnostic build (KS_LIB, tests/dev/devlib.py; e.g. the by-value merge_cl of commit
63524d5: make -C kubernetes-simulator_amd/csrc variant NAME=byval DEFS=-DKS_MCL_BYVAL) can be
compared bind for bind with the product.

    python tests/dev/byval_diag.py WORLD [FLAGS] OUT.npz"""
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402
_lib.LIB_PATH = lib_path(os.environ.get("KS_LIB", "libks_engine.so"))
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine, LocalExchange  # noqa: E402
import full_run_digest  # noqa: E402

world = int(sys.argv[1])
flags = int(sys.argv[2]) if len(sys.argv) > 2 else 0
out = sys.argv[3] if len(sys.argv) > 3 else None
g = full_run_digest.load("c5")
tr = tracegen.c5_trace(n_pods=g["pods"])
enc = encode.encode_trace(tr)
x = LocalExchange(world) if world > 1 else None
es = []
for r in range(world):
    e = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), engine_flags=flags)
    if world > 1:
        e.shard_host(world, r, x, 1)
    e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    e.submit(enc["pods"])
    es.append(e)
WATCH = int(os.environ.get("WATCH", "-1"))
if WATCH >= 0:
    es[0].debug_watch(WATCH)


def win_dtype():
    """ks_device.h WinWS of a -DKS_BATCH_LOG build, field for field (C alignment)."""
    B, S, R, E = 256, 512, 20, 2048
    return np.dtype([
        ("nb", "i4"), ("e_cnt", "i4"), ("n_e", "i4"), ("n_es", "i4"),
        ("win_hi", "i4", B), ("own", "i4", B), ("ex_q", "i4", S), ("ex_ok", "i4", S), ("ex_req", "i8", (S, 3)),
        ("e_node", "i4", E), ("e_off", "i4", S + 1), ("e_slot", "i4", S), ("e_rec", "u4", (E, 12)),
        ("cl_key", "u8", (B, R)), ("cl_info", "i4", B), ("cl_thr", "u8", B), ("cl_slot", "i4", (B, R)),
        ("nslot", "i4"), ("nslot_hw", "i4"), ("slot_node", "i4", B * R), ("slot_eix", "i4", 1536),
        ("slot_rec", "u4", (1536, 20)), ("touched", "i4", B + S), ("n_touched", "i4"), ("rescan", "i4"),
        ("lset", "i4"), ("pad_", "i4"),
        ("blog_n", "i4"), ("watch_pod", "i4"), ("watch_done", "i4"), ("wpad_", "i4"), ("blog", "i4", (16384, 4)),
        ("w_start", "i4"), ("w_nb", "i4"), ("w_c", "i4"), ("w_n_e", "i4"), ("w_n_es", "i4"), ("w_pad", "i4", 3),
        ("w_cl_key", "u8", (B, R)), ("w_cl_info", "i4", B), ("w_cl_thr", "u8", B), ("w_e_node", "i4", E),
        ("w_bind", "i4", B), ("w_adm", "i4", B)], align=True)


def show_watch(e, nodes_of_interest):
    raw = e.debug_window()
    dt = win_dtype()
    assert len(raw) == dt.itemsize, (len(raw), dt.itemsize)
    w = np.frombuffer(raw, dt)[0]
    n = int(w["blog_n"])
    lg = w["blog"][:min(n, 16384)]
    near = [tuple(int(x) for x in r) for r in lg if r[0] <= WATCH + 400 and r[0] + r[3] >= WATCH - 600]
    print(f"batches logged {n}; around pod {WATCH} (start, committed, stop, nb): {near}")
    if not w["watch_done"]:
        print("watched pod not recorded")
        return
    s0, nb, c = int(w["w_start"]), int(w["w_nb"]), int(w["w_c"])
    i = WATCH - s0
    E = set(int(x) for x in w["w_e_node"][:int(w["w_n_e"])])
    print(f"watch batch: start {s0} nb {nb} committed {c} n_e {int(w['w_n_e'])} (slot-E {int(w['w_n_es'])}); pod index {i} (chunk {i // 64})")
    info = int(w["w_cl_info"][i])
    keys = [int(k) for k in w["w_cl_key"][i][:info & 0xFF]]
    print(f"pod {WATCH}: info kept {info & 0xFF} trunc {bool(info & 256)} full {bool(info & 512)} ovf {bool(info & 1024)}; "
          f"thr total {int(w['w_cl_thr'][i]) >> 32} node {0xFFFFFFFF - (int(w['w_cl_thr'][i]) & 0xFFFFFFFF)}")
    print("   cl (node, total):", [(0xFFFFFFFF - (k & 0xFFFFFFFF), (k >> 32) - 1) for k in keys])
    for nd in nodes_of_interest:
        js = [s0 + j for j in range(c) if int(w["w_bind"][j]) == nd]
        print(f"   node {nd}: in E {nd in E}; binds in the batch at pods {js}")
    print("   batch binds before the pod:", [(s0 + j, int(w["w_bind"][j]), int(w["w_adm"][j])) for j in range(max(0, i - 8), i + 1)])


done = 0
nodes, stats = [], []
first_bad = None
for w, want in enumerate(g["bind_digests"]):
    k = min(g["window"], g["pods"] - done)
    res = [None] * world
    th = [threading.Thread(target=lambda r=r: res.__setitem__(r, es[r].step(k))) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    ok = [full_run_digest.bind_digest(b) == want for b in res]
    same = all(np.array_equal(res[0]["node"], b["node"]) and np.array_equal(res[0]["status"], b["status"]) for b in res)
    early = int(es[0].debug_counters()[4])
    inv = es[0].debug_invariants()
    print(f"window {w}: golden ok on ranks {sum(ok)}/{world}; ranks identical {same}; early stops {early}; {inv}", flush=True)
    if not same:
        for r in range(1, world):
            d = np.nonzero((res[0]["node"] != res[r]["node"]) | (res[0]["status"] != res[r]["status"]))[0]
            if len(d):
                print(f"   rank {r} differs from rank 0 first at pod {done + int(d[0])}", flush=True)
    if first_bad is None and not all(ok):
        first_bad = w
    if WATCH >= 0 and done <= WATCH < done + k:
        show_watch(es[0], [int(x) for x in os.environ.get("WATCH_NODES", "").split(",") if x])
    nodes.append(np.stack([b["node"] for b in res]))
    stats.append(np.stack([b["status"] for b in res]))
    done += k
if out:
    np.savez_compressed(out, nodes=np.concatenate(nodes, axis=1), status=np.concatenate(stats, axis=1))
print(f"first window off the golden: {first_bad}")
