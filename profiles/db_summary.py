"""Summaries of rocprofv3 result databases (ROCm 7.2 writes `run_results.db`, SQLite rocpd schema).

  python profiles/db_summary.py stats DB OUT.csv
      per-kernel dispatch statistics in rocprofv3's --stats CSV layout
  python profiles/db_summary.py timeline DB OUT.txt
      the batch chain as the GPU ran it: per kernel the average duration, per (kernel -> next kernel)
      pair the average idle gap between them, and the busy / idle split of the traced span
  python profiles/db_summary.py pmc FETCH_DB WRITE_DB SQ_DB OUT.json NOTE
      per-kernel averages of the PMC passes (profiles/collect.sh; SQ_DB may be ""); HBM bytes per launch =
      2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), the gfx950 correction of MI355X_MICROARCH.md §HBM
      (FETCH_SIZE tallies 128-B read requests at 64 B); SQ counters are summed over the shader
      engines of a dispatch, then averaged over dispatches
"""
import collections
import csv
import json
import sqlite3
import statistics
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].split("<")[0]


def stats(db, out):
    c = sqlite3.connect(db)
    rows = collections.defaultdict(list)
    for name, dur in c.execute("select name, duration from kernels"):
        rows[name].append(float(dur))
    total = sum(sum(v) for v in rows.values())
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v),
                        statistics.pstdev(v)])


def timeline(db, out):
    c = sqlite3.connect(db)
    ks = sorted((float(s), float(e), short(n)) for n, s, e in c.execute("select name, start, end from kernels"))
    dur = collections.defaultdict(list)
    gaps = collections.defaultdict(list)
    for i, (s, e, n) in enumerate(ks):
        dur[n].append(e - s)
        if i + 1 < len(ks):
            g = ks[i + 1][0] - e
            if g < 1e6:  # (host-side pauses between steps, > 1 ms, are not chain gaps)
                gaps[(n, ks[i + 1][2])].append(g)
    busy = sum(e - s for s, e, _ in ks)
    idle = sum(sum(v) for v in gaps.values())
    with open(out, "w") as f:
        f.write(f"kernels {len(ks)}, busy {busy / 1e6:.3f} ms, chain gaps {idle / 1e6:.3f} ms\n")
        for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
            f.write(f"  {n}: {len(v)} x {statistics.mean(v) / 1e3:.2f} us\n")
        f.write("gaps (kernel -> next): count x mean us\n")
        for (a, b), v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
            f.write(f"  {a} -> {b}: {len(v)} x {statistics.mean(v) / 1e3:.2f} us\n")


def per_kernel(db):
    """{kernel: {counter: mean over dispatches of the per-dispatch sum}}"""
    c = sqlite3.connect(db)
    acc = collections.defaultdict(float)
    for disp, kname, cname, val in c.execute(
            "select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        acc[(short(kname), cname, disp)] += float(val)
    sums = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, cn, _), v in acc.items():
        sums[k][cn].append(v)
    return {k: {cn: (sum(v) / len(v), len(v)) for cn, v in d.items()} for k, d in sums.items()}


def pmc(fetch_db, write_db, sq_db, out, note):
    f, w, s = per_kernel(fetch_db), per_kernel(write_db), (per_kernel(sq_db) if sq_db else {})
    res = {"source": note,
           "note": "HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), the gfx950 correction of "
                   "MI355X_MICROARCH.md §HBM; SQ_* summed over shader engines per dispatch "
                   "(SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_BUSY_CYCLES in quad-cycles), averaged over dispatches",
           "per_kernel": {}}
    for k in sorted(set(f) | set(w) | set(s)):
        d = {}
        if k in f:
            d["FETCH_SIZE_KB_avg"], d["launches"] = round(f[k]["FETCH_SIZE"][0], 1), f[k]["FETCH_SIZE"][1]
        if k in w:
            d["WRITE_SIZE_KB_avg"] = round(w[k]["WRITE_SIZE"][0], 1)
        for cn, (v, _) in sorted(s.get(k, {}).items()):
            d[cn + "_avg"] = round(v, 1)
        res["per_kernel"][k] = d
    scan = res["per_kernel"].get("ks::scan_kernel", {})
    if "FETCH_SIZE_KB_avg" in scan and "WRITE_SIZE_KB_avg" in scan:
        res["hbm_bytes_per_scan_launch"] = int((2 * scan["FETCH_SIZE_KB_avg"] + scan["WRITE_SIZE_KB_avg"]) * 1024)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "timeline":
        timeline(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "pmc":
        pmc(*sys.argv[2:7])
    else:
        raise SystemExit(__doc__)
