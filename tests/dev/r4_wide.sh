#!/bin/bash
# the chunk resolver on 32-bit words: resolver parity (incl. the wide instantiation), the C3q golden
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_resolvers_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_wide_parity.log 2>&1 || { tail -30 gpurun_out/r4_wide_parity.log; exit 1; }
tail -2 gpurun_out/r4_wide_parity.log
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu_config_size.py -x -q --timeout 300 --timeout-method thread -k c3q > gpurun_out/r4_c3q.log 2>&1 || { tail -30 gpurun_out/r4_c3q.log; exit 1; }
tail -2 gpurun_out/r4_c3q.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c5 --no-dropin > gpurun_out/r4_wide_bench.json 2>gpurun_out/r4_wide_bench.err || { tail gpurun_out/r4_wide_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4_wide_bench.json'));print('c3', d['pods_per_s']);print('c3q', d['c3q'])"
