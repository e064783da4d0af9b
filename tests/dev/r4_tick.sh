#!/bin/bash
# per-tick path: drop-in parity, the rate, a kernel trace of the per-tick run
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_dropin_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_tick_parity.log 2>&1 || { tail -30 gpurun_out/r4_tick_parity.log; exit 1; }
tail -2 gpurun_out/r4_tick_parity.log
timeout -k 10 300 python -u tests/dev/tick_rate.py > gpurun_out/r4_tick_rate.log 2>&1 || { tail gpurun_out/r4_tick_rate.log; exit 1; }
cat gpurun_out/r4_tick_rate.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_tick -o run -- python3 $GRAFT_REPO_ROOT/tests/dev/tick_rate.py > /dev/null 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/prof_tick -name "*kernel_stats.csv" | head -1 | xargs head -8
