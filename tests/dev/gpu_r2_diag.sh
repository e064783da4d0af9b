# dev: resolver-2 stamps diagnostic only
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tests/dev/diag_resolve2.py 256
