# Timing-only A/B of engine builds (no suite): C3 and C5 per-launch times, each build twice in
# alternating order, with a CRC of the binds (variants must match the base build's CRC).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for c in C3 C5; do
  for r in 1 2; do
    for v in "$@"; do
      timeout -k 10 150 python -u tests/dev/ab_scan.py $v $c 2>&1 | grep -v "^ *stopped" || exit 1
    done
  done
done
