set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sm_t.log 2>&1
rc=$?
tail -2 gpurun_out/sm_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 150 python -u tests/dev/diag_r4.py libks_engine_st.so || exit 1
bash tests/dev/ab_c4_only.sh libks_engine_base.so libks_engine.so libks_engine_base.so libks_engine.so
