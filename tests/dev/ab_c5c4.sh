# C5 and C4 A/B of engine builds (timing only; C5 kernel times with bind CRCs, C4 evals/s)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in "$@"; do
    timeout -k 10 150 python -u tests/dev/ab_scan.py $v C5 2>&1 | grep -v "^ *stopped" || exit 1
  done
done
bash tests/dev/ab_c4_pair.sh "$@"
