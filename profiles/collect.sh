#!/bin/bash
# Profile recipe for the committed summaries (run on the GPU box from the repo root):
#   bash profiles/collect.sh OUTDIR
# 1. rocprofv3 kernel trace + stats of the C3 bench (short) and of the C4 bench;
# 2. the PMC passes (one counter group per run): FETCH_SIZE, WRITE_SIZE, and the SQ instruction /
#    wave-cycle counters; 3. CSV / JSON summaries of the result databases (profiles/db_summary.py).
# Every step has its own time limit and the chain stops at the first failure.
set -euo pipefail
OUT=${1:-gpurun_out/prof}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
B="$ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/c3" -o run -- python3 $B > "$ROOT/$OUT/c3_bench.json"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/c4" -o run -- python3 "$ROOT/bench.py" --config c4 --steps 2 --warmup 1 > "$ROOT/$OUT/c4_bench.json"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$ROOT/$OUT/fetch" -o run -- python3 $B --steps 2 > /dev/null
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$ROOT/$OUT/write" -o run -- python3 $B --steps 2 > /dev/null
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$ROOT/$OUT/sq" -o run -- python3 $B --steps 2 > /dev/null
cd "$ROOT"
python3 profiles/db_summary.py stats "$OUT/c3/run_results.db" "$OUT/c3_kernel_stats.csv"
python3 profiles/db_summary.py stats "$OUT/c4/run_results.db" "$OUT/c4_kernel_stats.csv"
python3 profiles/db_summary.py pmc "$OUT/fetch/run_results.db" "$OUT/write/run_results.db" "$OUT/sq/run_results.db" \
    "$OUT/pmc_summary.json" "rocprofv3 --pmc passes over bench.py --steps 2 --warmup 1 (C3), MI355X"
echo "profiles collected in $OUT"
