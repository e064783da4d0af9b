"""The in-process all-gather behind ks_shard_host (include/ks_kubesim.h, ks_local_allgather): ranks
on threads of one process deposit their slices and each receives the rank-major concatenation —
over many consecutive exchanges (the engine calls it once per batch), with no GPU."""
import ctypes as C
import threading

import numpy as np

from kubesim_amd import _lib
from kubesim_amd.engine import LocalExchange


def _run(world, rounds, words):
    R = _lib.load_run()
    x = LocalExchange(world)
    bufs = [np.zeros(world * words, np.uint64) for _ in range(world)]
    errs = []

    def rank(r):
        for k in range(rounds):
            b = bufs[r]
            b[:] = 0
            b[r * words:(r + 1) * words] = (k << 32) | (r << 16) | np.arange(words, dtype=np.uint64)
            rc = R.ks_local_allgather(x.h, r, world, b.ctypes.data_as(C.c_void_p), 8 * words)
            want = np.concatenate([(k << 32) | (q << 16) | np.arange(words, dtype=np.uint64) for q in range(world)])
            if rc != 0 or not (b == want).all():
                errs.append((r, k, rc))
                return

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert not any(t.is_alive() for t in th), "exchange deadlocked"
    assert not errs, errs[:4]
    x.close()


def test_two_ranks_many_exchanges():
    _run(2, 300, 64)


def test_eight_ranks():
    _run(8, 50, 24)


def test_bad_arguments():
    R = _lib.load_run()
    x = LocalExchange(2)
    b = np.zeros(4, np.uint64)
    assert R.ks_local_allgather(x.h, 2, 2, b.ctypes.data_as(C.c_void_p), 16) == _lib.KS_EINVAL
    assert R.ks_local_allgather(x.h, 0, 3, b.ctypes.data_as(C.c_void_p), 16) == _lib.KS_EINVAL
