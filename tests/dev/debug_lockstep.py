import sys, numpy as np
sys.path[:0] = ['oracle', 'kubernetes-simulator_amd', 'tests']
from harness import small_trace, encoded, make_engine, make_oracle, MODES
from kubesim_amd.engine import KsError
for seed, mode, batch in ((1, "feeds_all_lrba", 0), (1, "feeds_all_lrba", 1), (1, "feeds_taint_sel_ba_const", 1)):
    tr = small_trace(seed, n_nodes=40, n_pods=160, arrival="stream")
    enc = encoded(tr)
    eng = make_engine(tr, enc, mode, batch); eng.submit(enc["pods"])
    ora = make_oracle(tr, mode); ora.submit(tr)
    for t in range(400):
        done = tr["pods"]["m"] - eng.queued
        fe, se = eng.filter(done) if done < 160 else None, eng.score(done) if done < 160 else None
        fo, so = ora.eval(done) if done < 160 else (None, None)
        try:
            eb = eng.step(1); erc = 0
        except KsError as e:
            eb = e.binds; erc = e.code; msg = str(e)
        ob, orc = ora.step(1)
        if len(eb) != len(ob['pod']) or erc != orc or (len(eb) and (eb['node'][0] != ob['node'][0] or eb['status'][0] != ob['status'][0])):
            print(seed, mode, batch, "tick", t+1, "done", done, "engine", eb, erc, (msg if erc else ''), "oracle", ob, orc)
            print(" eng filter", fe, "\n ora filter", fo, "\n eng score", se, "\n ora score", so)
            print(" pod tol/sel", hex(int(enc['pods']['tol'][done])), hex(int(enc['pods']['sel'][done])), "keymask", enc['pods']['keymask'][done])
            break
    else:
        print(seed, mode, batch, "ok")
