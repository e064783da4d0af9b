# New resolver: quick parity subset, then A/B timing against the role-split kernel, then the suite.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_quick.log 2>&1
rc=$?
echo "quick rc=$rc"; tail -15 gpurun_out/t_quick.log
if [ $rc -ne 0 ]; then exit $rc; fi
for c in C3 C5; do
  KS_RESOLVER=role timeout -k 10 150 python -u tests/dev/ab_scan.py libks_engine.so $c 2>&1 | sed 's/^/role  /' || exit 1
  timeout -k 10 150 python -u tests/dev/ab_scan.py libks_engine.so $c 2>&1 | sed 's/^/owner /' || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/t_suite.log 2>&1
rc=$?
echo "suite rc=$rc"; tail -5 gpurun_out/t_suite.log
