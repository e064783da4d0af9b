# C4 A/B of two builds (alternating, twice), then the full GPU suite with the in-tree build.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tests/dev/ab_c4_pair.sh "$@" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/t_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -5 gpurun_out/t_suite.log
exit $rc
