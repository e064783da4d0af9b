"""Benchmark: pod-node Filter+Score evals/s (and pods bound/s) of the HIP scheduling engine.

Workload (BASELINE.json configs[2], "C3"): 50,000 nodes with taints and labels, a 1M-pod
trace with tolerations / nodeSelectors / multi-phase simSpec, Filter (fit + taint +
selector) feeding Score (LeastRequested + BalancedAllocation), argmax, bind — one pod per
tick, in FIFO order, exactly the reference's loop (kubesim/kubesim.go:90-225).  Synthetic
data (tracegen, seed 0x5EED0003).

A "step" is one ks_step over --pods-per-step ticks (one bind per tick).  Every pod is
evaluated against every node (the reference's O(N) per pod), so evals = pods × nodes.
Inputs are resident on the device before the timed region (ks_submit_pods), the timed
region is K ks_step calls bracketed by a barrier + device synchronisation.

N > 1 (torchrun): every rank runs an independent what-if replica of the workload
(BASELINE.json configs[3] style: cluster replica × pod trace, seed ^ rank) on its own GPU;
no data-path collective — weak scaling; value = all ranks' evals ÷ the slowest rank's time.

Alongside (field "c5_sharded", every N): BASELINE.json configs[4] — one 1M-node cluster
node-sharded across the N ranks (ks_shard: each rank scans its node range, one RCCL all-gather
of the per-pod candidate lists per batch), total work fixed as N grows (strong scaling): the
north star's scaling target.  Skipped (with the reason) when ranks share a GPU.

roofline (roofline_block): the path is latency-bound (the resolver), so "achieved" / "frac" are
the MEASURED HBM bandwidth of a batch round (PMC bytes per round, profiles/pmc_<config>.json,
over its device time by HIP events) against 8 TB/s; the 80-B-per-evaluation model of SURVEY.md
§8(d) is "model_gbs" / "model_frac"; "stream_copy_gbs" is the HBM ceiling measured on the box.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-simulator_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BYTES_PER_EVAL = 80     # alloc[4] + reqTotal[3] + nRunning + taint + label


def _device(local_rank: int) -> int:
    """One rank per GPU; with fewer visible GPUs than ranks (a one-GPU rehearsal of N > 1) ranks
    share them round-robin.  torch.cuda.device_count() does not initialise the GPU."""
    try:
        import torch
        n = torch.cuda.device_count()
    except ImportError:
        n = 0
    return local_rank % n if n > 0 else local_rank


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _oracle_rate(trace, scorers, sample_pods, budget_s, threads):
    """(pods done, seconds) of the C oracle on the first pods of `trace` within `budget_s`."""
    import pyoracle
    from kubesim_amd import tracegen
    tr = tracegen.slice_pods(trace, 0, sample_pods)
    co = pyoracle.COracle(tr, filter_mode=1, filters=7, scorers=scorers)
    co.set_threads(threads)
    co.submit(tr)
    done, t0 = 0, time.perf_counter()
    while done < sample_pods and time.perf_counter() - t0 < budget_s:
        k = min(64, sample_pods - done)
        b, rc = co.step(k)
        done += k
        if rc:
            break
    dt = time.perf_counter() - t0
    co.close()
    return done, dt


def cpu_baseline(trace, scorers, sample_pods, budget_s):
    """The C oracle (faithful CPU restatement, SURVEY.md §8(d) CPU timing) on the first pods of
    the same trace on this host: (i) OpenMP over nodes on the host cores this job may use (the
    reported value) and (ii) single-threaded, each within `budget_s`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pyoracle.build()
    n = trace["nodes"]["n"]
    # the box exports OMP_NUM_THREADS = its CPU share; os.cpu_count() is the whole machine
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or min(os.cpu_count() or 1, 16)
    d_mt, t_mt = _oracle_rate(trace, scorers, sample_pods, budget_s, threads)
    d_st, t_st = _oracle_rate(trace, scorers, sample_pods, budget_s, 1)
    host = os.cpu_count() or 0
    return dict(value=d_mt * n / t_mt, unit="evals/s", cores=threads, kind="port",
                sample=f"C3 nodes ({n}), first {d_mt} pods of the trace, oracle/ks_oracle.c with OpenMP "
                       f"over nodes on {threads} threads ({t_mt:.1f} s)",
                cores_note=f"{threads} of the host's {host} hardware threads: the job's CPU share "
                           f"(OMP_NUM_THREADS on the GPU box; gpurun caps a job at 16), not the machine",
                pods_per_s=d_mt / t_mt,
                single_thread={"value": d_st * n / t_st, "pods_per_s": d_st / t_st, "cores": 1,
                               "sample": f"first {d_st} pods, one thread ({t_st:.1f} s)"})


def stream_copy_gbs(device: int, mib: int = 2048, reps: int = 10):
    """Measured HBM ceiling on this box: a device-to-device copy of `mib` MiB,
    read + write bytes over the time of `reps` copies (torch's copy kernel, HIP events)."""
    try:
        import torch
        if not torch.cuda.is_available():
            return None
        n = mib * (1 << 20) // 4
        a = torch.empty(n, dtype=torch.float32, device=f"cuda:{device}")
        b = torch.empty_like(a)
        a.fill_(1.0)
        b.copy_(a)
        torch.cuda.synchronize(device)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            b.copy_(a)
        t1.record()
        t1.synchronize()
        gbs = 2 * a.numel() * 4 * reps / (t0.elapsed_time(t1) * 1e-3) / 1e9
        del a, b
        torch.cuda.empty_cache()
        return round(gbs, 1)
    except Exception as ex:  # the measurement is informative only
        log(f"stream copy skipped: {ex}")
        return None


# the kernels of one batch round (rocprofv3 names -> roles of ks_kernel_stats).  The chunk
# resolver's chain (ks_step): window prep (a pass's first batch; an overlapped batch's window is
# computed inside the previous chunk kernel) -> scan (the overlap's conditional rescan, mostly an
# empty launch) -> merge with the candidate lists -> the chunk kernel, fused with the next batch's
# speculative scan and window prep ("fused") or alone ("resolve"); the small-cluster chain:
# expire_head -> scan -> merge -> resolve_kernel
BATCH_KERNELS = {"ks::expire_head_kernel": "prep", "ks::sq::window_prep_kernel": "prep",
                 "ks::scan_kernel": "scan", "ks::merge_kernel": "merge", "ks::merge_small_kernel": "merge",
                 "ks::sq::merge_cl_kernel": "merge",
                 "ks::resolve_kernel": "resolve", "ks::chk::resolve_chunk_kernel": "resolve",
                 "ks::chk::chunk_scan_kernel": "fused"}
VALU_ISSUE_PER_S = 256 * 4 * 0.5 * 2.4e9  # wave-instructions/s: 256 CUs x 4 SIMDs x 1/2 per cycle x 2.4 GHz


def load_pmc(config: str = "c3"):
    """Per-launch PMC averages of each batch kernel role from the committed summary of this workload
    (profiles/pmc_<config>.json, made by profiles/collect.sh + profiles/db_summary.py): HBM bytes =
    2 x FETCH_SIZE + WRITE_SIZE (the gfx950 correction of MI355X_MICROARCH.md §HBM), SQ_INSTS_VALU
    (wave-instructions, summed over the chip)."""
    p = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    per = {}
    for k, v in d.get("per_kernel", {}).items():
        role = BATCH_KERNELS.get(k)
        if not role:
            continue
        r = per.setdefault(role, {"bytes": 0, "valu": 0.0, "launches": 0})
        if "FETCH_SIZE_KB_avg" in v and "WRITE_SIZE_KB_avg" in v:
            r["bytes"] += int((2 * v["FETCH_SIZE_KB_avg"] + v["WRITE_SIZE_KB_avg"]) * 1024)
        r["valu"] += v.get("SQ_INSTS_VALU_avg", 0.0)
        r["launches"] += v.get("launches", 0)
    return {"per_role": per, "source": d.get("source", p), "file": os.path.relpath(p, ROOT)}


def usage_roofline(trace, kept, q_ticks, ku):
    """The per-tick usage kernel's roofline.  Algorithmic
    bytes of one query at tick t (§8(d)): per pod running at t, 16 B (node, t0, phase offset, phase
    count) + 4 B per phase scanned (the cumulative seconds up to its current phase) + 24 B of usage
    read + 24 B accumulated into its node — computed here from the binds and the trace.  achieved =
    those bytes / the kernel's HIP-event time (ks_last_step_kernels usage_ms / usage_n, the same ten
    queries); frac = achieved / 8,000 GB/s.  Beside it the committed PMC bytes of the kernel
    (profiles/pmc_c3.json "ks::usage_kernel": 2 x FETCH_SIZE + WRITE_SIZE, its own short run)."""
    import numpy as np
    if not ku.get("usage_n"):
        return None
    b = np.concatenate(kept)
    p = trace["pods"]
    tick = trace["tick_seconds"]
    off = p["phase_off"].astype(np.int64)
    sec = p["phase_sec"].astype(np.int64)
    q = b["pod"].astype(np.int64)
    tot = np.add.reduceat(sec, off[:-1])[q] if len(sec) else np.zeros(len(q), np.int64)
    tot = np.where(off[q + 1] > off[q], tot, 0)
    dur = -(-tot // tick)
    alg, nrun = [], []
    for t in q_ticks:
        run = (b["status"] == 0) & (b["tick"] <= t) & (t < b["tick"] + dur)
        nrun.append(int(run.sum()))
        nbytes = 0
        for j in np.nonzero(run)[0]:
            passed = (t - int(b["tick"][j])) * tick
            cs = np.cumsum(sec[off[q[j]]:off[q[j] + 1]])
            k = int(np.searchsorted(cs, passed, side="right"))  # first phase whose end is past `passed`
            nbytes += 16 + 4 * min(k + 1, len(cs)) + 24 + 24
        alg.append(nbytes)
    ms = ku["usage_ms"] / ku["usage_n"]
    a = float(np.mean(alg))
    achieved = a / (ms * 1e-3) / 1e9 if ms > 0 else None
    pmc = None
    pth = os.path.join(ROOT, "profiles", "pmc_c3.json")
    if os.path.exists(pth):
        with open(pth) as f:
            v = json.load(f).get("per_kernel", {}).get("ks::usage_kernel")
        if v and "FETCH_SIZE_KB_avg" in v and "WRITE_SIZE_KB_avg" in v:
            pmc = int((2 * v["FETCH_SIZE_KB_avg"] + v["WRITE_SIZE_KB_avg"]) * 1024)
    return {"bound": "latency (one small launch)", "kernel": "usage_kernel", "launch_ms": ms,
            "algorithmic_bytes": a, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None,
            "running_pods": float(np.mean(nrun)),
            "pods_read_per_launch": ku["usage_pods"] / ku["usage_n"], "traffic_pmc": pmc,
            "model": "per running pod 16 B + 4 B per phase scanned + 24 B usage read + 24 B node accumulate "
                     "(SURVEY.md 8(d)); the [N][3] zeroing and copy are outside the kernel"}


def roofline_block(value, st, ks, nodes, config, stream_gbs=None):
    """The roofline object: one formula, one configuration.

    Every time is a HIP-event average of the profiled step, which runs the same chain as the timed
    steps (the overlap on); every byte count is the committed PMC summary's per-launch average of
    the same kernel.  The dominant kernel is the batch kernel with the largest share of device time
    (C3: the resolve launch — the chunk kernel, fused with the next batch's scan and window prep on
    most batches, alone on a pass's last; C5 unsharded: the scan).  For it:
        traffic  = call-share-weighted PMC bytes per launch (2 x FETCH_SIZE + WRITE_SIZE)
        achieved = traffic / (its summed event ms / its launches)
        frac     = achieved / 8,000 GB/s
    beside it the algorithmic model (80 B per (pod, node) evaluation the launch performs, SURVEY.md
    §8(d): node records are reused across a scan workgroup's pods, so this exceeds the traffic),
    the scan's VALU-issue fraction (SQ_INSTS_VALU per launch / (1,024 SIMDs x 1/2 x 2.4 GHz x its
    time)) and the batch round (every kernel's time and bytes per batch)."""
    batches = max(st["launches"], 1)
    pods_per_batch = st["pods"] / batches
    pmc = load_pmc(config)
    per = pmc["per_role"] if pmc else {}
    roles = {"prep": (ks["prep_ms"], ks["prep_n"]), "scan": (ks["scan_ms"], ks["scan_n"]),
             "merge": (ks["merge_ms"], ks["merge_n"]),
             "resolve": (ks["resolve_ms"] + ks["fused_ms"], ks["resolve_n"] + ks["fused_n"])}
    dom = max(roles, key=lambda r: roles[r][0])
    ms_tot, n_dom = roles[dom]
    t_dom = ms_tot / max(n_dom, 1)
    if dom == "resolve":
        n_f, n_r = ks["fused_n"], ks["resolve_n"]
        b_f, b_r = (per.get("fused") or {}).get("bytes"), (per.get("resolve") or {}).get("bytes")
        traffic = (n_f * (b_f or 0) + n_r * (b_r or 0)) / max(n_f + n_r, 1) if (b_f or not n_f) and (b_r or not n_r) else None
        evals = pods_per_batch * nodes * n_f / max(n_f + n_r, 1)   # the fused scans' evaluations
        name = "resolve launch (chunk kernel; fused with the next batch's speculative scan + window prep)"
    else:
        b = (per.get(dom) or {}).get("bytes")
        traffic = b
        evals = pods_per_batch * nodes if dom == "scan" else 0
        name = dom
    achieved = traffic / (t_dom * 1e-3) / 1e9 if traffic and t_dom > 0 else None
    alg_gbs = BYTES_PER_EVAL * evals / (t_dom * 1e-3) / 1e9 if t_dom > 0 else None
    # the scan's VALU issue (standalone scan launches; at C3 with the overlap most are empty rescans,
    # the fused kernel's SQ_INSTS_VALU is reported with the resolve launch)
    t_scan = ks["scan_ms"] / max(ks["scan_n"], 1)
    v_scan = (per.get("scan") or {}).get("valu")
    v_fused = (per.get("fused") or {}).get("valu")
    t_fused = ks["fused_ms"] / max(ks["fused_n"], 1)
    round_ms = sum(v[0] for v in roles.values()) / batches
    round_bytes = sum((per.get(r) or {}).get("bytes", 0) * roles[r][1] for r in ("prep", "scan", "merge")) / batches
    round_bytes += ((per.get("fused") or {}).get("bytes", 0) * ks["fused_n"] +
                    (per.get("resolve") or {}).get("bytes", 0) * ks["resolve_n"]) / batches
    return {
        "bound": "latency" if dom == "resolve" else "VALU issue",
        "kernel": name,
        "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS if achieved is not None else None,
        "traffic": traffic,
        "formula": "frac = traffic / (event ms per launch) / 8000 GB/s; traffic = call-share-weighted PMC "
                   "(2 x FETCH_SIZE + WRITE_SIZE) per launch" + (f" from {pmc['file']}" if pmc else " (no PMC summary)"),
        "launch_ms": t_dom, "launches_per_batch": n_dom / batches,
        "algorithmic_bytes": BYTES_PER_EVAL * evals, "algorithmic_gbs": alg_gbs,
        "algorithmic_frac": alg_gbs / HBM_PEAK_GBS if alg_gbs is not None else None,
        "model": "80 B per (pod, node) evaluation the launch performs (SURVEY.md 8(d)); node records are "
                 "reused across a scan workgroup's pods (L2 / Infinity Cache), so it exceeds the traffic",
        "stream_copy_gbs": stream_gbs,
        "scan_valu_frac": v_scan / (VALU_ISSUE_PER_S * t_scan * 1e-3) if v_scan and t_scan > 0 else None,
        "fused_valu_frac": v_fused / (VALU_ISSUE_PER_S * t_fused * 1e-3) if v_fused and ks["fused_n"] else None,
        "batch_round": {
            "ms": round_ms, "pods": pods_per_batch, "hbm_bytes": round_bytes or None,
            "gbs": round_bytes / (round_ms * 1e-3) / 1e9 if round_bytes and round_ms > 0 else None,
            "kernels": {r: {"ms_per_launch": v[0] / max(v[1], 1), "launches_per_batch": v[1] / batches,
                            "hbm_bytes_per_launch": (per.get(r) or {}).get("bytes")}
                        for r, v in {**roles, "resolve": (ks["resolve_ms"], ks["resolve_n"]),
                                     "fused": (ks["fused_ms"], ks["fused_n"])}.items()},
        },
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods-per-step", type=int, default=32768)
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pods", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=0, help="pods per scan/resolve batch (0 = engine default: 192 on the chunk resolver)")
    ap.add_argument("--cpu-sample-pods", type=int, default=40000)
    ap.add_argument("--cpu-budget-s", type=float, default=12.0, help="per CPU-baseline leg (multi-core, single-thread)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", choices=("c3", "c4", "c5"), default="c3",
                    help="c3 (default): the metric's 50k-node workload; c4: BASELINE configs[3], "
                         "independent what-if scenarios batched in one launch per kernel; c5: "
                         "BASELINE configs[4], one 1M-node cluster node-sharded across the ranks")
    ap.add_argument("--scenarios", type=int, default=1024, help="c4: scenarios (split across ranks)")
    ap.add_argument("--scenario-nodes", type=int, default=2000)
    ap.add_argument("--scenario-pods", type=int, default=10_000)
    ap.add_argument("--c5-nodes", type=int, default=1 << 20)
    ap.add_argument("--c5-pods", type=int, default=100_000)
    ap.add_argument("--vshards", type=int, default=1, help="c5: virtual node shards per rank")
    ap.add_argument("--no-c5", action="store_true", help="c3: skip the C5 node-sharded leg")
    ap.add_argument("--no-dropin", action="store_true", help="c3: skip the drop-in Run-loop leg")
    ap.add_argument("--no-c3q", action="store_true", help="c3: skip the decimal-SI memory (C3q) leg")
    ap.add_argument("--no-c3-literal", action="store_true", help="c3: skip the reference-literal filter-mode leg")
    ap.add_argument("--no-c4", action="store_true", help="c3: skip the C4 what-if scenario leg")
    ap.add_argument("--c4-steps", type=int, default=2, help="c3: timed steps of the C4 leg")
    ap.add_argument("--c5-steps", type=int, default=4, help="c3: timed steps of the C5 leg")
    ap.add_argument("--c5-timeout", type=float, default=240.0,
                    help="c3: seconds the C5 leg may take before it is abandoned (the C3 line still prints)")
    args = ap.parse_args()
    if args.config == "c4":
        return main_c4(args)
    if args.config == "c5":
        return main_c5(args)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = _device(int(os.environ.get("LOCAL_RANK", "0")))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    from kubesim_amd import encode, tracegen
    from kubesim_amd.engine import Engine

    need = (args.steps + args.warmup) * args.pods_per_step
    n_pods = max(args.pods, need)
    seed = 0x5EED0003 ^ rank
    t0 = time.perf_counter()
    trace = tracegen.c3_trace(n_nodes=args.nodes, n_pods=n_pods, seed=seed)
    enc = encode.encode_trace(trace)
    scorers = ((1, 1, 0), (2, 1, 0))  # LeastRequested w1 + BalancedAllocation w1
    eng = Engine(tick_seconds=trace["tick_seconds"], filter_mode=1, filters=7, scorers=scorers,
                 device=local, batch_pods=args.batch)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    eng.submit(enc["pods"])
    log(f"[rank {rank}] trace {args.nodes} nodes x {n_pods} pods ready in {time.perf_counter() - t0:.1f}s")

    S = args.pods_per_step
    kept = []  # every step's binds (the usage kernel's algorithmic bytes need the placements)
    for _ in range(args.warmup):
        kept.append(eng.step(S))

    def barrier():
        # ks_step synchronises the engine's stream before returning; the extra device-wide
        # synchronize keeps the bracket honest if anything else were queued.
        if dist is not None:
            dist.barrier()
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize(local)
        except ImportError:
            pass

    barrier()
    t_start = time.perf_counter()
    binds = 0
    for _ in range(args.steps):
        b = eng.step(S)   # ks_step returns after its last kernel has completed
        binds += len(b)
        kept.append(b)
    t_el = time.perf_counter() - t_start
    barrier()
    if dist is not None:
        import torch
        t = torch.tensor([t_el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_el = float(t.item())
        c = torch.tensor([binds], dtype=torch.float64)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        total_binds = int(c.item())
    else:
        total_binds = binds

    # per-kernel breakdown on one more (profiled) step: HIP events on the engine's stream
    eng.set_profiling(True)
    kept.append(eng.step(S))
    st = eng.last_step_stats()
    kst = eng.last_step_kernels()
    eng.set_profiling(False)
    # per-tick node usage: ks_usage_at = zero + usage kernel over the pod
    # blocks that may run at t (run-interval index) + the [N][3] copy; the digest covers every
    # tick of the last step's window
    t_now = eng.tick
    eng.usage_at(t_now)
    t_u = time.perf_counter()
    q_ticks = [max(0, t_now - 1000 * k) for k in range(10)]
    for t_q in q_ticks:
        eng.usage_at(t_q)
    usage_ms = (time.perf_counter() - t_u) * 100.0
    # the usage kernel's roofline: the same ten queries with HIP events around the kernel alone
    eng.set_profiling(True)
    for t_q in q_ticks:
        eng.usage_at(t_q)
    ku = eng.last_step_kernels()
    eng.set_profiling(False)
    usage_roof = usage_roofline(trace, kept, q_ticks, ku)
    t_u = time.perf_counter()
    eng.usage_digest(max(0, t_now - S + 1), t_now + 1)
    digest_ms = (time.perf_counter() - t_u) * 1e3
    eng.close()
    dropin = dropin_leg(trace, enc, scorers, local) if rank == 0 and not args.no_dropin else None
    c3q = c3q_leg(args, scorers, local) if rank == 0 and not args.no_c3q else None
    c3lit = c3_literal_leg(args, trace, enc, scorers, local) if rank == 0 and not args.no_c3_literal else None
    # C4 (BASELINE configs[3]) on every rank: disjoint scenario ranges, weak scaling
    c4 = None
    if not args.no_c4:
        try:
            c4 = c4_leg(args, rank, world, local, dist)
        except Exception as ex:  # never fatal to the headline line on one rank
            if world > 1:
                # (a rank that skipped the leg's collectives would pair the C5 leg's
                # collectives with the other ranks' C4 ones — fail the run cleanly instead)
                raise
            log(f"[rank {rank}] C4 leg failed: {ex!r}")
            c4 = {"error": repr(ex)[:500]}
    line = None

    if rank == 0:
        nodes = args.nodes
        evals = total_binds * nodes
        value = evals / t_el
        pods_per_s = total_binds / t_el
        launches = max(st["launches"], 1)
        pods_per_launch = st["pods"] / launches
        scan_avg_ms = st["scan_ms"] / launches
        res_avg_ms = st["resolve_ms"] / launches
        other_avg_ms = st["other_ms"] / launches
        cpu = None
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N=1 figure
            cpu = cpu_baseline(trace, scorers, args.cpu_sample_pods, args.cpu_budget_s)
        line = {
            "metric": "pod-node Filter+Score evals/sec and pods bound/sec at 50k nodes, 1-8 GPUs",
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_el * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (tracegen C3, seed 0x5EED0003 ^ rank)",
            "config": {"workload": "C3: 50k nodes w/ taints+labels, 1M-pod trace, Filter(fit+taint+selector)"
                                   " -> Score(LR+BA) -> argmax -> bind, 1 pod/tick",
                       "nodes": nodes, "pods_per_step": S, "trace_pods": n_pods,
                       "parallelism": "replicas" if world > 1 else "single-gpu",
                       "batch_pods": args.batch or 192},
            "pods_per_s": pods_per_s,
            "roofline": roofline_block(value, st, kst, nodes, "c3", stream_copy_gbs(local)),
            "kernels": {"launches_per_step": launches, "pods_per_launch": pods_per_launch,
                        "scan_avg_ms": scan_avg_ms, "resolve_avg_ms": res_avg_ms,
                        "other_avg_ms": other_avg_ms,
                        "profiled_step_ms": st["step_ms"], "per_kernel": kst},
            "usage_query": {"ms_per_call": usage_ms, "nodes": nodes, "tick": t_now,
                            "digest_ms": digest_ms, "digest_ticks": S, "roofline": usage_roof,
                            "note": "ks_usage_at wall time at ticks near the end of the run, incl. the "
                                    "24 B/node copy to the host; digest = every tick of the last step's window"},
            "dropin": dropin,
            "c3q": c3q,
            "c3_literal": c3lit,
            "c4": c4,
            "c5_sharded": None,
            "cpu_baseline": cpu,
            "host": {"cpu": platform.processor() or platform.machine(), "nproc": os.cpu_count()},
        }
    if not args.no_c5:
        c5 = c5_leg(args, rank, world, local, dist, line=line)
        if rank == 0:
            line["c5_sharded"] = c5
    if rank == 0 and not line.get("_printed"):
        line["_printed"] = True
        print(json.dumps({k: v for k, v in line.items() if k != "_printed"}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def c3q_leg(args, scorers, device, steps=3, warmup=1, S=32768):
    """C3q: the C3 cluster and trace with decimal-SI memory requests on binary-SI
    capacities (tracegen.c3q_trace; the whole-run prefix is pinned by tests/golden/full_run.json
    "c3q").  The gcd of the memory quantities drops to 2^9: the node capacities scale past the micro
    evaluator's range.  Same timing bracket as the headline, fewer steps."""
    from kubesim_amd import encode, tracegen
    from kubesim_amd.engine import Engine
    n_pods = (steps + warmup + 1) * S
    tr = tracegen.c3q_trace(n_nodes=args.nodes, n_pods=1_000_000)
    tr = tracegen.slice_pods(tr, 0, n_pods)
    enc = encode.encode_trace(tr)
    eng = Engine(tick_seconds=tr["tick_seconds"], filter_mode=1, filters=7, scorers=scorers, device=device)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    eng.submit(enc["pods"])
    for _ in range(warmup):
        eng.step(S)
    t0 = time.perf_counter()
    binds = 0
    for _ in range(steps):
        binds += len(eng.step(S))
    dt = time.perf_counter() - t0
    eng.set_profiling(True)
    eng.step(S)
    st = eng.last_step_stats()
    eng.close()
    L = max(st["launches"], 1)
    return {"evals_per_s": binds * args.nodes / dt, "pods_per_s": binds / dt, "steps": steps, "pods_per_step": S,
            "pods_per_launch": st["pods"] / L, "scan_avg_ms": st["scan_ms"] / L,
            "resolve_avg_ms": st["resolve_ms"] / L, "other_avg_ms": st["other_ms"] / L,
            "workload": "C3q: C3 with decimal-SI memory requests on binary-SI capacities"}


def c3_literal_leg(args, trace, enc, scorers, device, steps=3, warmup=1, S=32768):
    """C3 in the reference's own filter mode: scheduleOneFilter's result is
    discarded (kubesim/kubesim.go:182), so every node is scored and admission alone decides Ok vs
    OverCapacity — the same trace and timing bracket as the headline, fewer steps.  The whole trace
    in this mode is pinned by tests/golden/full_run.json "c3lit"."""
    from kubesim_amd.engine import Engine
    eng = Engine(tick_seconds=trace["tick_seconds"], filter_mode=0, filters=7, scorers=scorers, device=device)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    eng.submit(enc["pods"])
    for _ in range(warmup):
        eng.step(S)
    t0 = time.perf_counter()
    binds, over = 0, 0
    for _ in range(steps):
        b = eng.step(S)
        binds += len(b)
        over += int((b["status"] == 1).sum())
    dt = time.perf_counter() - t0
    eng.set_profiling(True)
    eng.step(S)
    st = eng.last_step_stats()
    eng.close()
    L = max(st["launches"], 1)
    return {"evals_per_s": binds * args.nodes / dt, "pods_per_s": binds / dt, "steps": steps, "pods_per_step": S,
            "over_capacity_binds": over, "pods_per_launch": st["pods"] / L, "scan_avg_ms": st["scan_ms"] / L,
            "resolve_avg_ms": st["resolve_ms"] / L, "other_avg_ms": st["other_ms"] / L,
            "workload": "C3, reference-literal filter mode (kubesim.go:182: Filter result discarded), LR+BA"}


def dropin_leg(trace, enc, scorers, device, per_tick=4000, probe_ticks=400, windowed=65536, window=1024):
    """The drop-in's own call sequence on the C3 cluster with one pod arriving per tick.
    * native: KubeSim.Run / RunWindowed as a C++ host of the C-ABI (include/ks_kubesim.h,
      libks_kubesim.so) — per tick ks_submit_pods + ks_step(1) (the per-tick path: one launch), or
      `window` ticks of submits then one ks_step — the calls the Go shim makes through cgo
      (go/kubesim/engine/kubesim.go), with no interpreter between them;
    * python: the same loop through the Python twin (kubesim_amd.kubesim.KubeSim), plus the
      api.Filter / api.Scorer probe of the queue head (ks_filter + ks_score) every tick.
    Rates in pods/s (one pod binds per tick), wall time including every host call."""
    import numpy as np
    from kubesim_amd.engine import Engine
    from kubesim_amd.kubesim import KubeSim, NativeRun, TraceSubmitter, head_probe, slice_encoded

    def pods_of(n_pods):
        pods = dict(slice_encoded(enc["pods"], 0, n_pods))
        pods["arrival"] = np.arange(1, n_pods + 1, dtype=np.int64)
        return pods

    def engine():
        eng = Engine(tick_seconds=trace["tick_seconds"], filter_mode=1, filters=7, scorers=scorers, device=device)
        eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
        return eng

    out = {"workload": f"C3 cluster ({trace['nodes']['n']} nodes), trace pods 0.., one arrival per tick"}
    nr = NativeRun(engine(), pods_of(per_tick + 64), trace["tick_seconds"])
    nr.run(64)  # warm-up
    b, dt = nr.run(per_tick)
    out["per_tick"] = {"pods_per_s": len(b) / dt, "us_per_tick": dt / per_tick * 1e6, "ticks": per_tick,
                       "host": "C++ Run loop over the C-ABI (libks_kubesim.so)"}
    nr.eng.close()
    nr = NativeRun(engine(), pods_of(windowed + window), trace["tick_seconds"])
    nr.run(window, window)
    b, dt = nr.run(windowed, window)
    out["windowed"] = {"pods_per_s": len(b) / dt, "window": window, "ticks": windowed,
                       "host": "C++ RunWindowed over the C-ABI"}
    nr.eng.close()
    ks = KubeSim(engine(), trace["tick_seconds"])
    ks.register_submitter(TraceSubmitter(pods_of(per_tick + 64)))
    ks.run(64)
    t0 = time.perf_counter()
    ks.run(per_tick)
    dt = time.perf_counter() - t0
    out["python_per_tick"] = {"pods_per_s": per_tick / dt, "us_per_tick": dt / per_tick * 1e6, "ticks": per_tick}
    ks.eng.close()
    ks = KubeSim(engine(), trace["tick_seconds"])
    ks.register_submitter(TraceSubmitter(pods_of(probe_ticks + 16)))
    ks.run(16)
    t0 = time.perf_counter()
    ks.run(probe_ticks, probe=head_probe)
    dt = time.perf_counter() - t0
    out["python_per_tick_with_filter_score_probe"] = {"pods_per_s": probe_ticks / dt,
                                                      "us_per_tick": dt / probe_ticks * 1e6, "ticks": probe_ticks}
    ks.eng.close()
    return out


def main_c4(args):
    """--config c4: the C4 leg alone, printed as the line."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = _device(int(os.environ.get("LOCAL_RANK", "0")))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    line = c4_leg(args, rank, world, local, dist, steps=args.steps, warmup=args.warmup)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def c4_leg(args, rank, world, local, dist, steps=None, warmup=None):
    """BASELINE.json configs[3]: `scenarios` independent clusters (2k nodes, 10k-pod traces each,
    seed 0x5EED0004 ^ s) stepped together through ks_group_step; ranks take disjoint scenario
    ranges (weak scaling, no collective).  A step = `pods-per-step` ticks of every scenario (at most
    the trace / (steps + warmup)).  Part of the default run (the line's "c4" key)
    with 2 timed steps; --config c4 prints it alone.  Returns rank 0's dict (None elsewhere)."""
    from kubesim_amd import encode, tracegen
    from kubesim_amd.engine import Group
    steps = args.c4_steps if steps is None else steps
    warmup = 1 if warmup is None else warmup
    per = args.scenarios // world
    lo = rank * per
    S_pps = min(args.pods_per_step, args.scenario_pods // max(steps + warmup, 1))
    t0 = time.perf_counter()
    g = Group(per, device=local)
    scorers = ((1, 1, 0), (2, 1, 0))
    for s in range(lo, lo + per):
        tr = tracegen.c4_scenario(s, n_nodes=args.scenario_nodes, n_pods=args.scenario_pods)
        enc = encode.encode_trace(tr)
        e = g.add(tick_seconds=tr["tick_seconds"], filter_mode=1, filters=7, scorers=scorers, batch_pods=args.batch)
        e.load_nodes(enc["alloc"], enc["taint"], enc["label"])
        e.submit(enc["pods"])
    log(f"[rank {rank}] {per} scenarios ready in {time.perf_counter() - t0:.1f}s; {S_pps} ticks per step")
    for _ in range(warmup):
        g.step(S_pps)

    def barrier():
        if dist is not None:
            dist.barrier()
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize(local)
        except ImportError:
            pass

    barrier()
    t_start = time.perf_counter()
    binds, dev_ms, launches, aborted = 0, 0.0, 0, 0
    for k in range(steps):
        _, cnt, st, stats = g.step(S_pps)
        log(f"[rank {rank}] C4 step {k}: {stats['step_ms']:.1f} device ms, {stats['launches']} batch rounds")
        binds += int(cnt.sum())
        dev_ms += stats["step_ms"]
        launches += stats["launches"]
        aborted += sum(1 for x in st if x != 0)
    t_el = time.perf_counter() - t_start
    barrier()
    total = binds
    if dist is not None:
        import torch
        t = torch.tensor([t_el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_el = float(t.item())
        c = torch.tensor([binds], dtype=torch.float64)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        total = int(c.item())
    g.close()
    if rank != 0:
        return None
    evals = total * args.scenario_nodes
    return {
        "metric": "pod-node Filter+Score evals/sec and pods bound/sec (C4 what-if scenarios)",
        "value": evals / t_el, "unit": "evals/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": t_el * 1e3 / steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (tracegen C4, seed 0x5EED0004 ^ scenario)",
        "config": {"workload": "C4: independent what-if scenarios, Filter(fit+taint+selector) -> "
                               "Score(LR+BA) -> argmax -> bind per scenario, one launch per kernel",
                   "scenarios": per * world, "nodes_per_scenario": args.scenario_nodes,
                   "pods_per_scenario": args.scenario_pods, "ticks_per_step": S_pps,
                   "parallelism": f"scenarios/{world}"},
        "pods_per_s": total / t_el,
        "kernels": {"batch_rounds_per_step": launches / steps,
                    "device_ms_per_step": dev_ms / steps},
        "aborted_scenarios": aborted,
    }


def c5_leg(args, rank, world, local, dist, steps=None, warmup=1, line=None):
    """The C5 leg, never fatal to the bench line: an error on this rank is reported in rank 0's
    line.  A leg that hangs (e.g. a rank left waiting in an RCCL rendezvous) is ended by a
    watchdog after --c5-timeout s: rank 0 prints the C3 line with the leg marked abandoned (once)
    and every rank exits with status 3, so torchrun and the driver see the failure."""
    import threading
    timer = None
    if args.c5_timeout > 0:
        def _abandon():
            if rank == 0 and line is not None and not line.get("_printed"):
                line["c5_sharded"] = {"error": f"abandoned after {args.c5_timeout:.0f} s"}
                line["_printed"] = True
                print(json.dumps({k: v for k, v in line.items() if k != "_printed"}), flush=True)
            os._exit(3)
        timer = threading.Timer(args.c5_timeout, _abandon)
        timer.daemon = True
        timer.start()
    try:
        return _c5_leg_body(args, rank, world, local, dist, steps, warmup)
    except Exception as ex:  # e.g. an RCCL or HIP failure of a multi-rank run
        log(f"[rank {rank}] C5 leg failed: {ex!r}")
        return {"error": repr(ex)[:500]} if rank == 0 else None
    finally:
        if timer is not None:
            timer.cancel()


def _c5_leg_body(args, rank, world, local, dist, steps=None, warmup=1):
    """BASELINE.json configs[4]: one 1M-node cluster (tracegen C5, seed 0x5EED0005) node-sharded
    across the ranks — rank r scans its contiguous node range, the per-pod top-L candidate lists
    are all-gathered over RCCL once per batch, every rank resolves the same binds (ks_shard).
    Total work is fixed as N grows: strong scaling.  At N=1 the engine is unsharded unless
    --vshards > 1 (virtual shards on one GPU, the exchange without RCCL).  Returns rank 0's
    result dict (None on other ranks); a leg that cannot run says why."""
    steps = args.c5_steps if steps is None else steps
    if world > 1:
        try:
            import torch
            n_dev = torch.cuda.device_count()
        except ImportError:
            n_dev = 0
        if n_dev < world and not os.environ.get("KS_BENCH_SHARED_GPU"):  # rehearsal override
            return {"skipped": f"{world} ranks share {n_dev} GPU(s): RCCL needs one GPU per rank"}
    from kubesim_amd import encode, tracegen
    from kubesim_amd.engine import Engine, comm_unique_id
    need = (steps + warmup + 1) * args.pods_per_step
    n_pods = max(args.c5_pods, need)
    t0 = time.perf_counter()
    trace = tracegen.c5_trace(n_nodes=args.c5_nodes, n_pods=n_pods)
    enc = encode.encode_trace(trace)
    scorers = ((1, 1, 0), (2, 1, 0))
    eng = Engine(tick_seconds=trace["tick_seconds"], filter_mode=1, filters=7, scorers=scorers,
                 device=local, batch_pods=args.batch)
    if world > 1:
        idbox = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(idbox, src=0)
        eng.shard(world, rank, idbox[0], args.vshards)
    elif args.vshards > 1:
        eng.shard(1, 0, None, args.vshards)
    eng.load_nodes(enc["alloc"], enc["taint"], enc["label"])
    eng.submit(enc["pods"])
    del trace, enc
    log(f"[rank {rank}] C5 {args.c5_nodes} nodes x {n_pods} pods ready in {time.perf_counter() - t0:.1f}s")
    S = args.pods_per_step
    for _ in range(warmup):
        eng.step(S)

    def barrier():
        if dist is not None:
            dist.barrier()
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize(local)
        except ImportError:
            pass

    barrier()
    t_start = time.perf_counter()
    binds = 0
    for k in range(steps):
        binds += len(eng.step(S))
        log(f"[rank {rank}] C5 step {k} done")
    t_el = time.perf_counter() - t_start
    barrier()
    if dist is not None:
        import torch
        t = torch.tensor([t_el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_el = float(t.item())
    eng.set_profiling(True)
    eng.step(S)
    st = eng.last_step_stats()
    kst = eng.last_step_kernels()
    eng.set_profiling(False)
    eng.close()
    if rank != 0:
        return None
    nodes = args.c5_nodes
    launches = max(st["launches"], 1)
    return {
        "metric": "pod-node Filter+Score evals/sec and pods bound/sec (C5 1M-node sharded cluster)",
        "value": binds * nodes / t_el, "unit": "evals/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": t_el * 1e3 / steps, "scaling": "strong",
        "pods_per_s": binds / t_el,
        "data": "synthetic (tracegen C5, seed 0x5EED0005)",
        "config": {"workload": "C5: one 1M-node cluster, Filter(fit+taint+selector) -> Score(LR+BA) -> "
                               "argmax -> bind, node-sharded scan, per-batch RCCL candidate all-gather",
                   "nodes": nodes, "pods_per_step": S, "trace_pods": n_pods,
                   "parallelism": f"node-shards/{world}" + (f"x{args.vshards}v" if args.vshards > 1 else ""),
                   "batch_pods": args.batch or 192},
        "kernels": {"launches_per_step": launches, "pods_per_launch": st["pods"] / launches,
                    "scan_avg_ms": st["scan_ms"] / launches, "resolve_avg_ms": st["resolve_ms"] / launches,
                    "other_avg_ms": st["other_ms"] / launches, "profiled_step_ms": st["step_ms"],
                    "per_kernel": kst},
        "roofline": roofline_block(binds * nodes / t_el, st, kst, nodes, "c5"),
    }


def main_c5(args):
    """--config c5: the C5 leg alone, printed as the line."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = _device(int(os.environ.get("LOCAL_RANK", "0")))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    args.c5_timeout = 0
    line = c5_leg(args, rank, world, local, dist, steps=args.steps, warmup=args.warmup)
    if rank == 0:
        if "metric" not in line:  # the leg was skipped or failed: say so in a well-formed line
            line = {"metric": "pod-node Filter+Score evals/sec and pods bound/sec (C5 1M-node sharded cluster)",
                    "value": None, "unit": "evals/s", "n_gpus": world, "steps": args.steps,
                    "warmup": args.warmup, "scaling": "strong", **line}
        line.update({"higher_is_better": True, "vs_baseline": None, "dtype": "int64"})
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
