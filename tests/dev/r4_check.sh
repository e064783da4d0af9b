# New resolver: small GPU parity suite, then A/B timing of resolve_kernel (KS_RESOLVER=1) vs the
# register-table resolver (4) on C3 and C5 batches.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_t.log 2>&1
rc=$?
tail -5 gpurun_out/r4_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
for c in C3 C5; do
  for r in 1 4; do
    echo "KS_RESOLVER=$r"
    KS_RESOLVER=$r timeout -k 10 150 python -u tests/dev/ab_scan.py libks_engine.so $c || exit 1
  done
  for v in w8 np; do
    timeout -k 10 150 python -u tests/dev/ab_scan.py libks_engine_$v.so $c || exit 1
  done
done
