"""Timeline of a rocprofv3 kernel trace (run_results.db): per chunk-resolver launch, the time from
its start to the next one's start, how much of it the chunk kernel ran, and how much of each
speculative scan ran beside a chunk kernel (the overlap of ks_engine.cpp's step loop).
    python profiles/timeline.py DB [skip]"""
import collections
import sqlite3
import sys

db = sys.argv[1]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 50
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
qcol = next((x for x in ("stream_id", "queue_id", "queue") if x in cols), None)
rows = list(c.execute(f"select name, start, end{', ' + qcol if qcol else ''} from kernels order by start"))
short = lambda n: n.replace("void ", "").split("(")[0].split("<")[0]
ks = [(short(r[0]), int(r[1]), int(r[2]), r[3] if qcol else 0) for r in rows]
chunk = [k for k in ks if k[0].endswith("resolve_chunk_kernel")][skip:]
scans = [k for k in ks if k[0].endswith("scan_kernel")]
print("columns:", cols)
if len(chunk) < 3:
    sys.exit("too few chunk launches")
per = [(b[1] - a[1]) for a, b in zip(chunk, chunk[1:])]
dur = [a[2] - a[1] for a in chunk[:-1]]
print(f"chunk launches {len(chunk)}: start-to-start {sum(per) / len(per) / 1e3:.1f} us, chunk {sum(dur) / len(dur) / 1e3:.1f} us")
# per kind, mean duration and the mean time between the previous chunk's end and its start
names = collections.defaultdict(list)
for a, b in zip(chunk, chunk[1:]):
    for k in ks:
        if a[2] <= k[1] < b[1] or (a[1] <= k[1] < a[2] and k[0].endswith("scan_kernel")):
            names[k[0]].append((k[1] - a[2], k[2] - k[1], k[1] < a[2]))
for n, v in sorted(names.items()):
    inside = sum(1 for x in v if x[2])
    print(f"  {n:40s} n={len(v):5d} dur {sum(x[1] for x in v) / len(v) / 1e3:7.1f} us, "
          f"starts {sum(x[0] for x in v) / len(v) / 1e3:7.1f} us after the chunk end, {inside} started during a chunk")
# speculative scans: overlap with chunk kernels
ov, tot = 0, 0
for s in scans:
    tot += s[2] - s[1]
    for k in chunk:
        lo, hi = max(s[1], k[1]), min(s[2], k[2])
        if hi > lo:
            ov += hi - lo
print(f"scan time beside a chunk kernel: {ov / max(tot, 1) * 100:.1f} % of all scan time")
