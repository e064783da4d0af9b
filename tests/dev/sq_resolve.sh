set -e
export TMPDIR=/tmp
ROOT=$(pwd)
B="$ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline"
cd /tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$ROOT/gpurun_out/sq1" -o run -- python3 $B > /dev/null
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES -d "$ROOT/gpurun_out/sq2" -o run -- python3 $B > /dev/null
cd "$ROOT"
python3 - <<'PY'
import sqlite3, collections
for d in ("sq1","sq2"):
    c = sqlite3.connect(f"gpurun_out/{d}/run_results.db")
    acc = collections.defaultdict(float); n = collections.defaultdict(set)
    for disp, kn, cn, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        k = kn.split("(")[0].replace("void ","")
        if "resolve" not in k: continue
        acc[cn] += float(v); n[cn].add(disp)
    for cn in sorted(acc): print(d, cn, acc[cn] / len(n[cn]), "per launch over", len(n[cn]))
PY
