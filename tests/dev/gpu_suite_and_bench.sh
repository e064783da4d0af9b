set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/t_r2b.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/t_r2b.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/b_r2b.json 2> gpurun_out/b_r2b.log
echo "bench rc=$?"
cat gpurun_out/b_r2b.json
