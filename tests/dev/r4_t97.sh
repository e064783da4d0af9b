#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
for ov in 1 0; do echo "overlap=$ov"; KS_OVERLAP=$ov timeout -k 10 400 python -u -m pytest tests/test_engine_gpu_config_size.py -x -q --timeout 300 --timeout-method thread -k batch_independent 2>&1 | tail -3; done
