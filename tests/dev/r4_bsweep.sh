#!/bin/bash
# C3 bench at several batch sizes (the chunk class default is 192)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for bt in 192 160 224 256 192; do
  timeout -k 10 300 python -u bench.py --no-c5 --no-dropin --no-cpu-baseline --no-c3q --batch $bt > gpurun_out/bs_$bt.json 2> gpurun_out/bs_$bt.err || { tail -20 gpurun_out/bs_$bt.err; exit 1; }
  echo "batch=$bt $(python -c "import json; d=json.load(open('gpurun_out/bs_$bt.json')); print(d['value'], d['ms_per_step'])")"
done
