# owner-binds resolver: stamp breakdown (C3), then A/B timing against the role-split kernel.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tests/dev/diag_owner.py C3 || exit 1
for c in C3; do
  KS_RESOLVER=role timeout -k 10 150 python -u tests/dev/ab_scan.py libks_engine.so $c 2>&1 | sed 's/^/role  /' || exit 1
  timeout -k 10 150 python -u tests/dev/ab_scan.py libks_engine.so $c 2>&1 | sed 's/^/owner /' || exit 1
done
