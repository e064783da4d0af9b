"""Dev tool (not a test): the 2-rank x 4-part C5 run of tests/test_shard_world_gpu.py with a logging
exchange (a Python callback around ks_local_allgather) and a watchdog, to see where a hang sits:
in the exchange (a rank waiting for the other's deposit) or on the device.
    python tests/dev/pipe_hang.py WORLD VSH [FLAGS]"""
import ctypes as C
import faulthandler
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from kubesim_amd import _lib, encode, tracegen  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
_lib.LIB_PATH = lib_path(os.environ.get("KS_LIB", "libks_engine.so"))
from kubesim_amd.engine import Engine, LocalExchange  # noqa: E402
import full_run_digest  # noqa: E402

world, vsh = int(sys.argv[1]), int(sys.argv[2])
flags = int(sys.argv[3]) if len(sys.argv) > 3 else 0
faulthandler.dump_traceback_later(50, exit=True)
g = full_run_digest.load("c5")
tr = tracegen.c5_trace(n_pods=g["pods"])
enc = encode.encode_trace(tr)
x = LocalExchange(world)
R = _lib.load_run()
FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int64)
calls = [0] * world
t0 = time.time()


@FN
def logged(user, rank, w, buf, nbytes):
    calls[rank] += 1
    if calls[rank] <= 3 or calls[rank] % 200 == 0:
        print(f"  [{time.time() - t0:6.2f}s] rank {rank} exchange #{calls[rank]} ({nbytes} B) in", flush=True)
    rc = R.ks_local_allgather(x.h, rank, w, buf, nbytes)
    return rc


def watchdog():  # a rank waiting for a partner that never comes: abort the exchange, then compare logs
    last = list(calls)
    while True:
        time.sleep(3)
        if calls == last and not all_done[0]:
            print(f"[{time.time() - t0:6.2f}s] no exchange progress: {calls}; aborting", flush=True)
            R.ks_local_exchange_abort(x.h)
            return
        last = list(calls)


all_done = [False]


class _X:
    fn = C.cast(logged, C.c_void_p)
    h = None


es = []
for r in range(world):
    e = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), engine_flags=flags)
    e.shard_host(world, r, _X(), vsh)
    e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    e.submit(enc["pods"])
    es.append(e)
threading.Thread(target=watchdog, daemon=True).start()
done = 0
for w, want in enumerate(g["bind_digests"]):
    k = min(g["window"], g["pods"] - done)
    res = [None] * world
    def run(r):
        try:
            res[r] = es[r].step(k)
        except Exception as ex:  # noqa: BLE001
            res[r] = ex
    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if any(isinstance(b, Exception) for b in res):
        print(f"window {w}: aborted {res}", flush=True)
        if os.environ.get("KS_LIB", "").endswith("blog.so"):
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from winws import win_dtype
            logs = []
            for r in range(world):
                wv = np.frombuffer(es[r].debug_window(), win_dtype())[0]
                logs.append([tuple(int(v) for v in row) for row in wv["blog"][:min(int(wv["blog_n"]), 16384)]])
            n = min(len(l) for l in logs)
            first = next((i for i in range(n) if logs[0][i] != logs[1][i]), None)
            print(f"batches logged per rank {[len(l) for l in logs]}; first differing batch {first}", flush=True)
            if first is not None:
                for r in range(world):
                    print(f"  rank {r}: {logs[r][max(0, first - 3):first + 3]}", flush=True)
        break
    ok = [full_run_digest.bind_digest(b) == want for b in res]
    print(f"[{time.time() - t0:6.2f}s] window {w}: golden ok {sum(ok)}/{world}; exchanges {calls}", flush=True)
    done += k
print("done")
