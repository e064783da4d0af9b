#!/bin/bash
# round-4 evidence: GPU suite, smoke, bench line, chunk phase breakdown, profiles (collect.sh)
set -o pipefail
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04/gpu_suite.log 2>&1
rc=$?; tail -3 gpurun_out/r04/gpu_suite.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.log 2>&1 || { tail gpurun_out/r04/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r04/bench.json 2> gpurun_out/r04/bench.err || { tail gpurun_out/r04/bench.err; exit 1; }
timeout -k 10 300 python -u tests/dev/diag_chunk.py > gpurun_out/r04/chunk_phase_breakdown.txt 2>&1 || exit 1
bash profiles/collect.sh gpurun_out/r04 > gpurun_out/r04/collect.log 2>&1 || { tail -20 gpurun_out/r04/collect.log; exit 1; }
echo done
