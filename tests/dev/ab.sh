#!/bin/bash
# Diagnostic A/B timing of engine builds on the C3 resolver workload (GPU box):
#   tests/dev/ab.sh libA.so libB.so ...   -> gpurun_out/ab.log
mkdir -p gpurun_out
: > gpurun_out/ab.log
for L in "$@"; do
  echo "== $L" >> gpurun_out/ab.log
  KS_DIAG_LIB=$L timeout -k 10 100 python tests/dev/diag_resolve.py 256 2>&1 | grep -E "^B=|resolve |stopped|warmup" >> gpurun_out/ab.log || true
done
