set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 150 python -u tests/dev/diag_r4.py libks_engine_st.so
