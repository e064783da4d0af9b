#!/bin/bash
# round 4: the chunk resolver on candidate slots in the fused chain: parity, then timing
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_resolvers_gpu.py tests/test_engine_gpu.py tests/test_engine_gpu_c2.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r4_chunk_parity.log 2>&1
rc=$?
tail -5 gpurun_out/r4_chunk_parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tests/dev/ab_resolvers.py chunk chunk@256 > gpurun_out/r4_chunk_ab.log 2>&1 || exit $?
cat gpurun_out/r4_chunk_ab.log
