# Timing A/B of engine builds (C3 / C5 per-launch kernel times, bind CRCs), then the full GPU suite
# and the default + C4 bench lines with the in-tree build.   bash tests/dev/ab_suite_bench.sh A.so B.so
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in C3 C5; do
  for v in "$@"; do
    timeout -k 10 150 python -u tests/dev/ab_scan.py $v $c 2>&1 | grep -v "^ *stopped" || exit 1
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/t_suite.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/t_suite.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/t_suite.log | head -20; exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/b_c3.json 2> gpurun_out/b_c3.log
rc=$?
echo "bench rc=$rc"
cat gpurun_out/b_c3.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.log
echo "c4 rc=$?"
cat gpurun_out/b_c4.json
