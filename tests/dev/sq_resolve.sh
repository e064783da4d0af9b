# SQ instruction / wait counters of the resolve kernel on the C3 bench (two PMC passes), per launch;
# summary in gpurun_out/sq_resolve.txt, databases removed (they exceed gpurun's copy-back limit).
set -e
export TMPDIR=/tmp
ROOT=$(pwd)
LIBV=${1:-}
B="$ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5"
cd /tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d /tmp/sq1 -o run -- python3 $B > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -d /tmp/sq2 -o run -- python3 $B > /dev/null 2>&1
cd "$ROOT"
mkdir -p gpurun_out
python3 - <<'PY' | tee gpurun_out/sq_resolve.txt
import sqlite3, collections
for d in ("sq1", "sq2"):
    c = sqlite3.connect(f"/tmp/{d}/run_results.db")
    acc = collections.defaultdict(float); n = collections.defaultdict(set)
    q = ("select d.dispatch_id, k.kernel_name, p.counter_name, p.value from counters_collection p "
         "join kernel_dispatch d using(dispatch_id) join kernel_symbols k using(kernel_id)")
    try:
        rows = list(c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"))
    except Exception:
        rows = list(c.execute(q))
    for disp, kn, cn, v in rows:
        if "resolve_kernel" not in kn:
            continue
        acc[cn] += float(v); n[cn].add(disp)
    for cn in sorted(acc):
        print(d, cn, round(acc[cn] / len(n[cn]), 1), "per launch over", len(n[cn]))
PY
rm -rf /tmp/sq1 /tmp/sq2
