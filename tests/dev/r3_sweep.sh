# Round 3: resolver parity (all forced resolvers) + C3 whole-trace golden per resolver, then A/B.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_resolvers_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t_res.log 2>&1
rc=$?; echo "resolvers rc=$rc"; tail -4 gpurun_out/t_res.log
if [ $rc -ne 0 ]; then grep -B5 -A40 "FAILED\|Error" gpurun_out/t_res.log | head -80; exit $rc; fi
timeout -k 10 600 python -u -m pytest "tests/test_engine_gpu_config_size.py::test_c3_whole_trace_matches_oracle_golden" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_c3g.log 2>&1
rc=$?; echo "c3 golden rc=$rc"; tail -4 gpurun_out/t_c3g.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tests/dev/ab_resolvers.py one_pod sweep sweep:8 sweep:16 > gpurun_out/ab_res.txt 2>&1
rc=$?; cat gpurun_out/ab_res.txt; exit $rc
