# Round 3 evidence: GPU suite, smoke, default bench line, then the rocprof kernel stats + PMC
# passes (profiles/collect.sh) into gpurun_out/prof_r03.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1
rc=$?; tail -3 gpurun_out/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/b_r3.json 2> gpurun_out/b_r3.log
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('gpurun_out/b_r3.json')); print(d['value'], d['pods_per_s'], d['ms_per_step'], d['c5_sharded']['value'])"
SKIP_C4=1 bash profiles/collect.sh gpurun_out/prof_r03
