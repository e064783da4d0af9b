# C4 A/B: two engine builds, alternating, twice each (timing only)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for v in "$@"; do
    echo "== $v"; timeout -k 10 200 python -u tests/dev/ab_c4.py $v 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels'])" || exit 1
  done
done
