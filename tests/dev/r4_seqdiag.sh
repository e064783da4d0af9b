#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
KS_DIAG_LIB=libks_engine_seqdiag.so timeout -k 10 300 python -u tests/dev/ab_resolvers.py seq > gpurun_out/r4_seq_diag.log 2>&1 || exit $?
cat gpurun_out/r4_seq_diag.log
