# C4 evals/s at several batch sizes (timing only)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for b in 0 96 64; do
    echo "== batch $b"
    timeout -k 10 200 python -u bench.py --config c4 --steps 2 --warmup 1 --batch $b 2>/dev/null | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels'])" || exit 1
  done
done
