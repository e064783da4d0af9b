"""Dev tool (not a test): ks_device.h WinWS of a -DKS_BATCH_LOG diagnostic build as a numpy dtype
(C alignment, field for field), and a printer of the watched pod's batch (ks_debug_watch)."""
import numpy as np


def win_dtype():
    B, S, R, E = 256, 512, 20, 2048
    return np.dtype([
        ("nb", "i4"), ("e_cnt", "i4"), ("n_e", "i4"), ("n_es", "i4"),
        ("win_hi", "i4", B), ("own", "i4", B), ("ex_q", "i4", S), ("ex_ok", "i4", S), ("ex_req", "i8", (S, 3)),
        ("e_node", "i4", E), ("e_off", "i4", S + 1), ("e_slot", "i4", S), ("e_rec", "u4", (E, 12)),
        ("cl_key", "u8", (B, R)), ("cl_info", "i4", B), ("cl_thr", "u8", B), ("cl_slot", "i4", (B, R)),
        ("nslot", "i4"), ("nslot_hw", "i4"), ("slot_node", "i4", B * R), ("slot_eix", "i4", 1536),
        ("slot_rec", "u4", (1536, 20)), ("touched", "i4", B + S), ("n_touched", "i4"), ("rescan", "i4"),
        ("lset", "i4"), ("pad_", "i4"), ("split", "i4"), ("moff", "i4"), ("mpar", "i4"), ("pad2_", "i4"),
        ("mrg", "u8", (2, B, 12)),
        ("blog_n", "i4"), ("watch_pod", "i4"), ("watch_done", "i4"), ("wpad_", "i4"), ("blog", "i4", (16384, 4)),
        ("w_start", "i4"), ("w_nb", "i4"), ("w_c", "i4"), ("w_n_e", "i4"), ("w_n_es", "i4"), ("w_pad", "i4", 3),
        ("w_cl_key", "u8", (B, R)), ("w_cl_info", "i4", B), ("w_cl_thr", "u8", B), ("w_e_node", "i4", E),
        ("w_bind", "i4", B), ("w_adm", "i4", B), ("w_nsw", "i4"), ("w_pad2", "i4"), ("w_dec", "i4", (64, 8)),
        ("w_smeta", "i2", (64, 8)), ("w_rowcid", "i4", 64)], align=True)


def show_watch(e, watch, nodes_of_interest=()):
    raw = e.debug_window()
    dt = win_dtype()
    assert len(raw) == dt.itemsize, (len(raw), dt.itemsize)
    w = np.frombuffer(raw, dt)[0]
    n = int(w["blog_n"])
    lg = w["blog"][:min(n, 16384)]
    near = [tuple(int(x) for x in r) for r in lg if r[0] <= watch + 400 and r[0] + r[3] >= watch - 600]
    print(f"batches logged {n}; around pod {watch} (start, committed, stop, nb): {near}")
    if not w["watch_done"]:
        print("watched pod not recorded")
        return
    s0, nb, c = int(w["w_start"]), int(w["w_nb"]), int(w["w_c"])
    i = watch - s0
    E = set(int(x) for x in w["w_e_node"][:int(w["w_n_e"])])
    print(f"watch batch: start {s0} nb {nb} committed {c} n_e {int(w['w_n_e'])} (slot-E {int(w['w_n_es'])}); "
          f"pod index {i} (chunk {i // 64})")
    info = int(w["w_cl_info"][i])
    keys = [int(k) for k in w["w_cl_key"][i][:info & 0xFF]]
    print(f"pod {watch}: info kept {info & 0xFF} trunc {bool(info & 256)} full {bool(info & 512)} ovf {bool(info & 1024)}; "
          f"thr total {(int(w['w_cl_thr'][i]) >> 32) - 1} node {0xFFFFFFFF - (int(w['w_cl_thr'][i]) & 0xFFFFFFFF)}")
    print("   cl (node, total):", [(0xFFFFFFFF - (k & 0xFFFFFFFF), (k >> 32) - 1) for k in keys])
    for nd in nodes_of_interest:
        js = [s0 + j for j in range(c) if int(w["w_bind"][j]) == nd]
        print(f"   node {nd}: in E {nd in E}; binds in the batch at pods {js}")
    print("   binds before the pod (pod, node, adm):",
          [(s0 + j, int(w["w_bind"][j]), int(w["w_adm"][j])) for j in range(max(0, i - 8), min(i + 1, c))])
    ns = int(w["w_nsw"])
    print(f"   sweeps deciding the pod: {ns}")
    for k in range(min(ns, 64)):
        f, lo, bad, code, nw, dc, dkt, c0 = (int(x) for x in w["w_dec"][k])
        print(f"     fresh {f} lo {lo} bad {bad} code {code} winner cid {nw} D cid {dc} D total {dkt - 1} (c0 {c0})")
    print("   chunk rows at the chunk's end (row: seg starts, ovf, cid | guess cid):")
    for r in range(64):
        m = [int(x) for x in w["w_smeta"][r]]
        if m[6] >= 0:
            print(f"     row {r}: segs {m[:5]} ovf {m[5]} cid {m[6]} | guess {int(w['w_rowcid'][r])}")
