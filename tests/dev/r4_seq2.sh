#!/bin/bash
# round 4: sequential resolver parity (forced) + chunk vs seq A/B on C3 and C5 + diag counters
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_resolvers_gpu.py -x -q --timeout 300 --timeout-method thread -k "seq" > gpurun_out/r4_seq_parity.log 2>&1
rc=$?
tail -5 gpurun_out/r4_seq_parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tests/dev/ab_resolvers.py chunk seq seq@192 > gpurun_out/r4_seq_ab.log 2>&1 || exit $?
cat gpurun_out/r4_seq_ab.log
KS_DIAG_LIB=libks_engine_seqdiag.so timeout -k 10 300 python -u tests/dev/ab_resolvers.py seq > gpurun_out/r4_seq_diag.log 2>&1 || exit $?
cat gpurun_out/r4_seq_diag.log
timeout -k 10 300 python -u tests/dev/ab_resolvers.py --c5 chunk seq > gpurun_out/r4_seq_ab_c5.log 2>&1 || exit $?
cat gpurun_out/r4_seq_ab_c5.log
