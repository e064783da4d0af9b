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


def test_abort_releases_waiting_ranks():
    """A rank that failed before its deposit: its driver aborts the exchange and the ranks already
    waiting in it (and any later call) return KS_EDEVICE instead of hanging."""
    R = _lib.load_run()
    x = LocalExchange(3)
    rcs = {}

    def rank(r):
        b = np.zeros(3 * 4, np.uint64)
        rcs[r] = R.ks_local_allgather(x.h, r, 3, b.ctypes.data_as(C.c_void_p), 32)

    th = [threading.Thread(target=rank, args=(r,)) for r in (0, 1)]  # rank 2 never arrives
    for t in th:
        t.start()
    import time
    time.sleep(0.2)
    assert all(t.is_alive() for t in th)  # both wait for rank 2
    x.abort()
    for t in th:
        t.join(10)
    assert not any(t.is_alive() for t in th), "abort did not release the waiting ranks"
    assert rcs == {0: _lib.KS_EDEVICE, 1: _lib.KS_EDEVICE}
    b = np.zeros(12, np.uint64)
    assert R.ks_local_allgather(x.h, 2, 3, b.ctypes.data_as(C.c_void_p), 32) == _lib.KS_EDEVICE
    x.close()
