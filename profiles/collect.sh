#!/bin/bash
# Profile recipe for the committed summaries (run on the GPU box from the repo root):
#   bash profiles/collect.sh OUTDIR
# 1. rocprofv3 kernel trace + stats of the C3 bench (short, the line's own chain: overlap on; with the
#    batch chain's per-kernel durations and gaps, db_summary.py timeline), the C4 bench and the C5 bench;
# 2. the PMC passes (one counter group per run): FETCH_SIZE, WRITE_SIZE, and the SQ instruction /
#    wave-cycle counters, for C3 and C5; 3. CSV / JSON summaries of the result databases
#    (profiles/db_summary.py).  Every step has its own time limit and the chain stops at the first
#    failure.
set -euo pipefail
OUT=${1:-gpurun_out/prof}
ROOT=$(pwd)
DB=/tmp/ks_prof   # result databases (large): scratch, summaries go to OUT
mkdir -p "$OUT" "$DB"
export TMPDIR=/tmp
# heartbeat under OUT (a profiled run prints nothing for minutes; gpurun takes silence for a hang)
( while true; do date +%T >> "$OUT/heartbeat.txt"; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
B="$ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-c5 --no-dropin --no-c3q --no-c4 --no-c3-literal"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$DB/c3" -o run -- python3 $B > "$ROOT/$OUT/c3_bench.json"
echo "c3 trace done"
if [ -z "${SKIP_C4:-}" ]; then
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$DB/c4" -o run -- python3 "$ROOT/bench.py" --config c4 --steps 2 --warmup 1 > "$ROOT/$OUT/c4_bench.json"
echo "c4 trace done"
fi
# PMC passes serialise every dispatch: a short step (8,192 pods, ~45 batch rounds) keeps each pass
# within its limit; the summaries are per-launch averages
P="$B --steps 1 --pods-per-step 8192"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$DB/fetch" -o run -- python3 $P > /dev/null
echo "fetch pass done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$DB/write" -o run -- python3 $P > /dev/null
echo "write pass done"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$DB/sq" -o run -- python3 $P > /dev/null
echo "sq pass done"
C5="$ROOT/bench.py --config c5 --steps 2 --warmup 1"
if [ -z "${SKIP_C5:-}" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$DB/c5" -o run -- python3 $C5 > "$ROOT/$OUT/c5_bench.json"
echo "c5 trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$DB/c5fetch" -o run -- python3 $C5 --steps 1 --warmup 0 > /dev/null
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$DB/c5write" -o run -- python3 $C5 --steps 1 --warmup 0 > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d "$DB/c5sq" -o run -- python3 $C5 --steps 1 --warmup 0 > /dev/null
echo "c5 pmc done"
fi
cd "$ROOT"
if [ -z "${SKIP_C5:-}" ]; then
python3 profiles/db_summary.py stats "$DB/c5/run_results.db" "$OUT/c5_kernel_stats.csv"
python3 profiles/db_summary.py pmc "$DB/c5fetch/run_results.db" "$DB/c5write/run_results.db" "$DB/c5sq/run_results.db" \
    "$OUT/pmc_c5.json" "rocprofv3 --pmc passes over bench.py --config c5 --steps 1 --warmup 0 (C5, 1M nodes), MI355X"
fi
python3 profiles/db_summary.py stats "$DB/c3/run_results.db" "$OUT/c3_kernel_stats.csv"
python3 profiles/db_summary.py timeline "$DB/c3/run_results.db" "$OUT/c3_timeline.txt"
[ -z "${SKIP_C4:-}" ] && python3 profiles/db_summary.py stats "$DB/c4/run_results.db" "$OUT/c4_kernel_stats.csv"
python3 profiles/db_summary.py pmc "$DB/fetch/run_results.db" "$DB/write/run_results.db" "$DB/sq/run_results.db" \
    "$OUT/pmc_c3.json" "rocprofv3 --pmc passes over bench.py --steps 1 --warmup 1 --pods-per-step 8192 (C3 alone), MI355X"
rm -rf "$DB"
echo "profiles collected in $OUT"
