# Round 3: the GPU suite (small tests first, then the config-size ones), stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_small.log 2>&1
rc=$?; echo "small rc=$rc"; tail -5 gpurun_out/t_small.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; echo "all rc=$rc"; tail -5 gpurun_out/t_all.log
exit $rc
