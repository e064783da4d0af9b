# A/B of resolver build variants (product lib, then each KS_DIAG_LIB variant), then stamps of each.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ab.txt
for lib in "" $AB_LIBS; do
  echo "== lib ${lib:-libks_engine.so}" >> gpurun_out/ab.txt
  KS_DIAG_LIB=$lib timeout -k 10 200 python -u tests/dev/ab_pair.py >> gpurun_out/ab.txt 2>&1 || { cat gpurun_out/ab.txt; exit 1; }
done
for lib in $STAMP_LIBS; do
  echo "== stamps $lib" >> gpurun_out/ab.txt
  KS_DIAG_LIB=$lib timeout -k 10 200 python -u tests/dev/diag_pair.py >> gpurun_out/ab.txt 2>&1 || { cat gpurun_out/ab.txt; exit 1; }
done
cat gpurun_out/ab.txt
