# Round 3: default bench line (C3 + C5 leg + drop-in leg), one-pod vs pair resolver A/B on C3 / C5.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/b_r3.json 2> gpurun_out/b_r3.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/b_r3.json
exit $rc
