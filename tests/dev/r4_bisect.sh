#!/bin/bash
set -o pipefail
export PYTHONUNBUFFERED=1
for ov in 0 1; do echo "overlap=$ov"; KS_OVERLAP=$ov timeout -k 10 300 python -u tests/dev/bisect_batch.py 0 97 || exit 1; done
