# A/B of two engine builds on C3 / C5 (kernel times, bind CRCs) and C4 (evals/s), then the suite.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in C3 C5; do
  for v in "$@"; do
    timeout -k 10 150 python -u tests/dev/ab_scan.py $v $c 2>&1 | grep -v "^ *stopped" || exit 1
  done
done
bash tests/dev/ab_c4_pair.sh "$@" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/t_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -5 gpurun_out/t_suite.log
exit $rc
