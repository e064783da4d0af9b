#!/bin/bash
# round 4: the per-tick path + native Run loop, host-exchange ranks, the sequential resolver's
# parity suite, then chunk vs seq on C3 (timing + diag counters)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_dropin_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r4_dropin.log 2>&1
rc=$?
tail -25 gpurun_out/r4_dropin.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_resolvers_gpu.py -x -v --timeout 300 --timeout-method thread -k "seq" > gpurun_out/r4_seq_parity.log 2>&1
rc=$?
tail -5 gpurun_out/r4_seq_parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tests/dev/ab_resolvers.py chunk seq seq@192 > gpurun_out/r4_seq_ab.log 2>&1 || exit $?
cat gpurun_out/r4_seq_ab.log
KS_DIAG_LIB=libks_engine_seqdiag.so timeout -k 10 300 python -u tests/dev/ab_resolvers.py seq > gpurun_out/r4_seq_diag.log 2>&1 || exit $?
cat gpurun_out/r4_seq_diag.log
timeout -k 10 600 python -u -m pytest tests/test_shard_world_gpu.py -x -v --timeout 500 --timeout-method thread > gpurun_out/r4_world.log 2>&1
rc=$?
tail -8 gpurun_out/r4_world.log
exit $rc
