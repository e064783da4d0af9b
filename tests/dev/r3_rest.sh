# Round 3: the rest of the GPU suite (C4 golden, large, usage/keys), drop-in rates, then the bench.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_usage_keys_gpu.py tests/test_dropin_gpu.py -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/t_rest.log 2>&1
rc=$?; echo "rest rc=$rc"; tail -4 gpurun_out/t_rest.log; grep "drop-in" gpurun_out/t_rest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/b_r3.json 2> gpurun_out/b_r3.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b_r3.json
exit $rc
