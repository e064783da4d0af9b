set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for r in 1 4; do
  echo "KS_RESOLVER=$r"
  KS_RESOLVER=$r timeout -k 10 200 python -u bench.py --config c4 --steps 2 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('pods_per_s'), d.get('kernels'))" || exit 1
done
