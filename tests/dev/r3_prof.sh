# Round 3: pair-resolver stamp breakdown, then the profile recipe into gpurun_out/prof_r03.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tests/dev/diag_pair.py > gpurun_out/diag_pair.txt 2>&1
rc=$?; echo "diag rc=$rc"; cat gpurun_out/diag_pair.txt
if [ $rc -ne 0 ]; then exit $rc; fi
bash profiles/collect.sh gpurun_out/prof_r03
