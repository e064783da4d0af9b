# Default bench line, then the profile recipe (profiles/collect.sh) into gpurun_out/prof_r2g.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/b_r2g.json 2> gpurun_out/b_r2g.log
rc=$?
echo "bench rc=$rc"
if [ $rc -ne 0 ]; then tail -20 gpurun_out/b_r2g.log; exit $rc; fi
bash profiles/collect.sh gpurun_out/prof_r2g
