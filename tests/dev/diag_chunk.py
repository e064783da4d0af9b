"""Diagnostic: chunk-resolver counters (`make chunkdiag`, -DKS_CHUNK_DIAG) on the C3 bench workload.
ctr[5] launches, [6] pods committed, [7] sweeps, [8] chunks, [9..14] early stops by reason (0 unknown
state / both cached nodes rebound, 1 candidate buffer overflow, 2 truncated list, 3 exhausted list,
4 admission unknown, 5 NotFound / bad pod), [16..20] cycles: setup, per-chunk cache, sweeps,
finalize, commit; [21] cids, [22] E nodes, [23] batch pods."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from devlib import lib_path  # noqa: E402
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
from kubesim_amd import _lib
_lib.LIB_PATH = lib_path(os.environ.get("KS_DIAG_LIB", "libks_engine_chunkdiag.so"))
from kubesim_amd import tracegen, encode
from kubesim_amd.engine import Engine
c5 = "--c5" in sys.argv
tr = tracegen.c5_trace(n_pods=120_000) if c5 else tracegen.c3_trace(n_pods=200_000)
enc = encode.encode_trace(tr)
eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), engine_flags=64)
eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
eng.submit(enc["pods"])
if "--noprof" not in sys.argv:  # (profiling times each kernel: no overlap)
    eng.set_profiling(True)
eng.step(32768)
c0 = eng.debug_counters().copy()
t = time.perf_counter(); eng.step(32768); dt = time.perf_counter() - t
st = eng.last_step_stats()
d = eng.debug_counters() - c0
L = max(d[5], 1)
print(f"launches {L}, pods/launch {d[6] / L:.1f} (batch {d[23] / L:.1f}), sweeps/launch {d[7] / L:.1f}, chunks/launch {d[8] / L:.2f}, "
      f"cids {d[21] / L:.0f}; wall {32768 / dt:.0f} pods/s")
print("early stops by reason (row state unknown, buf ovf, trunc, exhausted, adm unknown or notfound/bad, "
      "cached state unknown, both cached rebound):", [int(x) for x in d[9:14]] + [int(d[14]), int(d[22])])
print("cycles per launch: setup %.0f, cache %.0f, sweeps %.0f (%.0f per sweep), finalize %.0f, commit %.0f" % (
    d[16] / L, d[17] / L, d[18] / L, d[18] / max(d[7], 1), d[19] / L, d[20] / L))
if "--d2" in sys.argv:  # (make chunkdiag DIAGLVL=2 NAME=2: d[24..31] remapped)
    print("cache per chunk with c0 > 0 (%.2f per launch): rebase %.0f, slot replays %.0f, top two %.0f, reduce %.0f cycles" % (
        (d[8] - L) / L, *(d[24 + q] / max(d[8] - L, 1) for q in range(4))))
    print("commit %.0f = replays %.0f + rest; tail window prep %.0f; setup loads to first barrier %.0f cycles per launch" % (
        d[20] / L, d[28] / L, d[30] / L, d[31] / L))
    sys.exit(0)
print("exclusion-only rounds/launch %.1f; phases, cycles per round (both kinds): A marks %.0f, B replay %.0f, C decide %.0f, D converge %.0f" % ((d[28] / L,) + tuple(d[24 + q] / max(d[7] + d[28], 1) for q in range(4))))
print("phase C per exclusion-only round %.0f, per full sweep %.0f cycles; B per full sweep %.0f" % (d[15] / max(d[28], 1), d[26] / max(d[7], 1), d[25] / max(d[7], 1)))
print("phase C split per full sweep (wave 0, C1 and entries / rows / cached D + reduce): %.0f / %.0f / %.0f cycles" % (
    d[29] / max(d[7], 1), d[30] / max(d[7], 1), d[31] / max(d[7], 1)))
nl = max(st["launches"], 1)
print(f"resolve {st['resolve_ms'] / nl * 1e3:.1f} us/launch (prep + cl + chunk kernels), scan {st['scan_ms'] / nl * 1e3:.1f}, other {st['other_ms'] / nl * 1e3:.1f}")
