set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_engine_gpu_c5.py -x -q --timeout 200 --timeout-method thread > gpurun_out/thr_t.log 2>&1
rc=$?
tail -3 gpurun_out/thr_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tests/dev/ab_scan_only.sh libks_engine_base.so libks_engine.so || exit 1
for v in libks_engine_base.so libks_engine.so; do
  echo "C4 $v"
  timeout -k 10 200 python -u tests/dev/ab_c4.py $v 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels'])" || exit 1
done
