#!/bin/bash
# persistent scan on C5: the C5 goldens, then the C5 bench line and its kernel trace
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu_c5.py tests/test_engine_gpu_config_size.py tests/test_shard_world_gpu.py -x -q --timeout 600 --timeout-method thread -k "c5 or world" > gpurun_out/r4_c5_parity.log 2>&1 || { tail -30 gpurun_out/r4_c5_parity.log; exit 1; }
tail -2 gpurun_out/r4_c5_parity.log
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/r4_c5_bench.json 2> gpurun_out/r4_c5_bench.err || { tail gpurun_out/r4_c5_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4_c5_bench.json'));print(d['pods_per_s'], d['kernels'])"
