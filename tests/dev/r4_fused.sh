#!/bin/bash
# fused chunk + speculative scan: parity, the batch-independence test, A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_resolvers_gpu.py tests/test_engine_gpu.py tests/test_dropin_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_fu_parity.log 2>&1 || { tail -30 gpurun_out/r4_fu_parity.log; exit 1; }
tail -2 gpurun_out/r4_fu_parity.log
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu_config_size.py -x -q --timeout 600 --timeout-method thread -k "not c4" > gpurun_out/r4_fu_golden.log 2>&1 || { tail -30 gpurun_out/r4_fu_golden.log; exit 1; }
tail -2 gpurun_out/r4_fu_golden.log
for ov in 0 1; do KS_OVERLAP=$ov timeout -k 10 300 python -u tests/dev/ab_resolvers.py --noprof chunk > gpurun_out/r4_fu_ab$ov.log 2>&1 || exit 1; echo "overlap=$ov"; cat gpurun_out/r4_fu_ab$ov.log; done
