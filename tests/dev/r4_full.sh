#!/bin/bash
# round 4: the whole GPU suite, smoke, then the default bench line
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_gpu_suite.log 2>&1
rc=$?
tail -4 gpurun_out/r4_gpu_suite.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/r4_gpu_suite.log | head -20; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -20 gpurun_out/r4_smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || { tail -20 gpurun_out/r4_bench.err; exit 1; }
cat gpurun_out/r4_bench.json
