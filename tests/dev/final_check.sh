# Final check of the committed build: the full GPU suite, smoke(), the default bench line.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/t_final.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -3 gpurun_out/t_final.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/b_final.json 2> gpurun_out/b_final.log
rc=$?
echo "bench rc=$rc"
python -c "import json; d=json.load(open('gpurun_out/b_final.json')); print(d['value'], d['pods_per_s'], d['roofline']['frac'], d['c5_sharded'].get('value'))"
exit $rc
