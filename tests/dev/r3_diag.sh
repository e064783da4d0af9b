set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tests/dev/ab_pair.py > gpurun_out/ab_pair.txt 2>&1
rc=$?; cat gpurun_out/ab_pair.txt; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tests/dev/diag_pair.py > gpurun_out/diag_pair.txt 2>&1
rc=$?; cat gpurun_out/diag_pair.txt; exit $rc
