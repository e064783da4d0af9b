"""Dev tool (not a test): the terms of the 8-GPU C5 batch time, measured on one GPU.

Rank 0 of an 8-rank node-sharded engine (ks_shard_host, world 8) on the C5 cluster: it scans only
its 512 blocks (1/8 of the 1M nodes) and, with the overlap, fuses that scan into its chunk kernel —
exactly what each of 8 ranks would run — while the exchange is a host callback that leaves the other
ranks' parts empty (their candidates are missing, so the binds differ from a real run; the kernels'
work per batch is the same: every list of this rank's range is merged and every pod resolved).
Prints the per-kernel HIP-event times of a profiled step (ks_last_step_kernels) and the same for the
unsharded engine (T(1)).  The RCCL all-gather's own time is not measured (one GPU)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib  # noqa: E402
_lib.LIB_PATH = lib_path(os.environ.get("KS_LIB", "libks_engine.so"))
from kubesim_amd import encode, tracegen  # noqa: E402
from kubesim_amd.engine import Engine  # noqa: E402

S = 32768
WORLD = int(os.environ.get("T8_WORLD", "8"))
tr = tracegen.c5_trace(n_pods=4 * S)
enc = encode.encode_trace(tr)
FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int64)


@FN
def lone_exchange(user, rank, world, buf, bytes_per_rank):
    # the other ranks' slices: empty lists (zero keys)
    for r in range(world):
        if r != rank:
            C.memset(buf + r * bytes_per_rank, 0, bytes_per_rank)
    return 0


class _X:  # what Engine.shard_host expects of an exchange
    fn = C.cast(lone_exchange, C.c_void_p)
    h = None


def run(world, flags=0):
    eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), engine_flags=flags)
    if world > 1:
        eng.shard_host(world, 0, _X(), 1)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    eng.submit(enc["pods"])
    eng.step(S)
    c0 = eng.debug_counters()
    eng.step(S)  # unprofiled: the batch time as the bench runs it (HIP events around the whole step)
    st0 = eng.last_step_stats()
    c1 = eng.debug_counters()
    eng.set_profiling(True)
    eng.step(S)
    st, k = eng.last_step_stats(), eng.last_step_kernels()
    eng.close()
    nb = max(st["launches"], 1)
    us = lambda ms, n: ms / max(n, 1) * 1e3  # noqa: E731
    print(f"world {world} flags {flags}: {st0['step_ms'] / max(st0['launches'], 1) * 1e3:.1f} us per batch "
          f"({st['step_ms'] / nb * 1e3:.1f} profiled), {st0['pods'] / max(st0['launches'], 1):.1f} pods/batch; "
          f"per step: {st0['launches']} batches, {int(c1[4])} early stops, {int(c1[5] - c0[5])} rescans, "
          f"{int(c1[6] - c0[6])} list reuses")
    print(f"   prep {us(k['prep_ms'], k['prep_n']):.1f} us x {k['prep_n'] / nb:.2f}, scan {us(k['scan_ms'], k['scan_n']):.1f}, "
          f"merge {us(k['merge_ms'], k['merge_n']):.1f} (part merges {us(k['part_ms'], k['xchg_n']):.1f}, "
          f"host exchange {us(k['xchg_ms'], k['xchg_n']):.1f} x {k['xchg_n'] / nb:.2f}), resolve {us(k['resolve_ms'], k['resolve_n']):.1f} x "
          f"{k['resolve_n'] / nb:.2f}, fused {us(k['fused_ms'], k['fused_n']):.1f} x {k['fused_n'] / nb:.2f}")
    if k["side_n"]:
        print(f"   pipelined: main-stream wait for the exchange {us(k['wait_ms'], nb):.1f} us per batch; second stream "
              f"per batch: speculative scan {us(k['side_scan_ms'], k['side_n']):.1f}, part merges "
              f"{us(k['side_part_ms'], k['side_n']):.1f}, exchange {us(k['side_xchg_ms'], k['side_n']):.1f}")


run(1)
run(WORLD)
run(WORLD, _lib.KS_ENGINE_NO_OVERLAP)
