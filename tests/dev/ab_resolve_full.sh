# The whole GPU suite on the current build, then C3 / C5 per-launch times of the builds named
# on the command line (A/B), then the stamps breakdown.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/abf_t.log 2>&1
rc=$?
tail -3 gpurun_out/abf_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
for c in C3 C5; do
  for v in "$@"; do
    timeout -k 10 150 python -u tests/dev/ab_scan.py $v $c || exit 1
  done
done
timeout -k 10 200 python -u tests/dev/diag_resolve.py 256
