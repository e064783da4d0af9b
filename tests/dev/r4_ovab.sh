#!/bin/bash
# overlap A/B only (wall rate + CRC), C3 and C5
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for ov in 0 1; do KS_OVERLAP=$ov timeout -k 10 300 python -u tests/dev/ab_resolvers.py --noprof chunk > gpurun_out/r4_ov_ab$ov.log 2>&1 || exit 1; echo "overlap=$ov"; cat gpurun_out/r4_ov_ab$ov.log; done
for ov in 0 1; do KS_OVERLAP=$ov timeout -k 10 300 python -u tests/dev/ab_resolvers.py --noprof --c5 chunk > gpurun_out/r4_ov_c5_$ov.log 2>&1 || exit 1; echo "c5 overlap=$ov"; cat gpurun_out/r4_ov_c5_$ov.log; done
