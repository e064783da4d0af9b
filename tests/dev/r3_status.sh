# Round 3 status: resolver A/B on C3 and C5, then the GPU suite, then the default bench line.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tests/dev/ab_resolvers.py one_pod pair sweep > gpurun_out/ab_c3.txt 2>&1
rc=$?; cat gpurun_out/ab_c3.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/dev/ab_resolvers.py --c5 one_pod pair sweep > gpurun_out/ab_c5.txt 2>&1
rc=$?; cat gpurun_out/ab_c5.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1
rc=$?; tail -5 gpurun_out/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/b_r3.json 2> gpurun_out/b_r3.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b_r3.json; exit $rc
