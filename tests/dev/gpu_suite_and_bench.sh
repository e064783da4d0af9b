# Full GPU suite, the default bench line and the C4 line.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/t_r2c.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/t_r2c.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/b_r2c.json 2> gpurun_out/b_r2c.log
rc=$?
echo "bench rc=$rc"
cat gpurun_out/b_r2c.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/c4_r2c.json 2> gpurun_out/c4_r2c.log
echo "c4 rc=$?"
cat gpurun_out/c4_r2c.json
