set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  echo "C4 $v"
  timeout -k 10 200 python -u tests/dev/ab_c4.py $v 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernels'])" || exit 1
done
