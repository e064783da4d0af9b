#!/bin/bash
# static candidates per pod (KS_CHR variants, make variant NAME=r16 DEFS=-DKS_CHR=16): C3 bench, interleaved
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do for v in "" _r16 _r20; do
  KS_LIB=libks_engine$v.so timeout -k 10 300 python -u tests/dev/ab_lib.py --no-c5 --no-dropin --no-cpu-baseline > gpurun_out/chr$v.json 2> gpurun_out/chr$v.err || { tail -20 gpurun_out/chr$v.err; exit 1; }
  echo "[$v] $(python -c "import json; d=json.load(open('gpurun_out/chr$v.json')); print(d['value'], d['ms_per_step'], d['c3q']['pods_per_s'])")"
done; done
