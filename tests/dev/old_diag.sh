set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tests/dev/diag_resolve.py 256
