# Full GPU suite, the default bench line, and the C4 A/B of the register-table resolver's pruning.
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
for v in libks_engine.so libks_engine_np.so; do
  echo "C4 $v"
  timeout -k 10 200 python -u tests/dev/ab_c4.py $v 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels'])" || exit 1
done
