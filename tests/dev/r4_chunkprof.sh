#!/bin/bash
# chunk on slots: quick parity, A/B, and a rocprofv3 kernel trace of the bench's C3 steps
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_resolvers_gpu.py -x -q --timeout 300 --timeout-method thread -k chunk > gpurun_out/r4_chunk_parity.log 2>&1 || { tail -30 gpurun_out/r4_chunk_parity.log; exit 1; }
tail -2 gpurun_out/r4_chunk_parity.log
timeout -k 10 300 python -u tests/dev/ab_resolvers.py chunk > gpurun_out/r4_chunk_ab.log 2>&1 || exit $?
cat gpurun_out/r4_chunk_ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_chunk -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-c5 --no-dropin > $GRAFT_REPO_ROOT/gpurun_out/r4_prof_bench.log 2>&1 || exit $?
find $GRAFT_REPO_ROOT/gpurun_out/prof_chunk -name "*kernel_stats.csv" | head -1 | xargs head -12
