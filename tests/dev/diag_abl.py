"""Diagnostic: time resolver ablation builds (results invalid by construction; timing only).
usage: python tests/dev/diag_abl.py [lib-suffix ...]   (runs each in its own process)"""
import os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIBDIR = os.path.join(ROOT, "kubernetes-simulator_amd", "kubesim_amd")

def one(suffix, B):
    sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))
    from kubesim_amd import _lib
    _lib.LIB_PATH = os.path.join(LIBDIR, f"libks_engine{suffix}.so")
    from kubesim_amd import tracegen, encode
    from kubesim_amd.engine import Engine
    tr = tracegen.c3_trace(n_pods=200_000)
    enc = encode.encode_trace(tr)
    eng = Engine(tick_seconds=10, filter_mode=1, filters=7, scorers=((1, 1, 0), (2, 1, 0)), batch_pods=B)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    eng.submit(enc["pods"])
    eng.step(65536)
    eng.set_profiling(True)
    c0 = eng.debug_counters().copy()
    t = time.perf_counter(); eng.step(32768); dt = time.perf_counter() - t
    st = eng.last_step_stats()
    d = eng.debug_counters() - c0
    print(f"{suffix or 'base':8s} wall {dt*1e3:7.1f} ms  {dt/32768*1e6:6.2f} us/pod  launches {st['launches']}"
          f"  early {d[4]}  resolve {st['resolve_ms']:.1f} ms", flush=True)

if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        one(sys.argv[2] if sys.argv[2] != "base" else "", int(sys.argv[3]))
        sys.exit(0)
    B = int(os.environ.get("B", "256"))
    for suf in (sys.argv[1:] or ["base"]):
        r = subprocess.run([sys.executable, __file__, "--one", suf, str(B)], timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)
