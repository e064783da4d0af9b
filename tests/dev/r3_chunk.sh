# Round 3: chunk resolver parity (forced, every resolver case), C3 golden with it, then A/B.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_resolvers_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k chunk > gpurun_out/t_chunk.log 2>&1
rc=$?; echo "chunk resolvers rc=$rc"; tail -4 gpurun_out/t_chunk.log
if [ $rc -ne 0 ]; then grep -B5 -A60 "FAILED\|Error\|error" gpurun_out/t_chunk.log | head -120; exit $rc; fi
timeout -k 10 300 python -u tests/dev/ab_resolvers.py one_pod chunk > gpurun_out/ab_chunk.txt 2>&1
rc=$?; cat gpurun_out/ab_chunk.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest "tests/test_engine_gpu_config_size.py::test_c3_whole_trace_matches_oracle_golden[chunk]" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_c3g.log 2>&1
rc=$?; echo "c3 golden rc=$rc"; tail -4 gpurun_out/t_c3g.log; exit $rc
