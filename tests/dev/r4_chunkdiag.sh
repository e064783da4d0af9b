#!/bin/bash
# chunk resolver: parity, A/B timing and the per-phase cycle counters (chunkdiag build)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_resolvers_gpu.py -x -q --timeout 300 --timeout-method thread -k chunk > gpurun_out/r4_chunk_parity.log 2>&1 || { tail -30 gpurun_out/r4_chunk_parity.log; exit 1; }
tail -2 gpurun_out/r4_chunk_parity.log
timeout -k 10 300 python -u tests/dev/ab_resolvers.py chunk > gpurun_out/r4_chunk_ab.log 2>&1 || exit $?
cat gpurun_out/r4_chunk_ab.log
timeout -k 10 300 python -u tests/dev/diag_chunk.py > gpurun_out/r4_chunk_diag.log 2>&1 || exit $?
cat gpurun_out/r4_chunk_diag.log
