set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for c in C3 C5; do
  for v in "$@"; do
    timeout -k 10 150 python -u tests/dev/ab_scan.py $v $c 2>&1 | grep -v "^ *stopped" || exit 1
  done
done
