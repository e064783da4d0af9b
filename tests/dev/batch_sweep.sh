set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bs_t.log 2>&1
rc=$?
tail -2 gpurun_out/bs_t.log
if [ $rc -ne 0 ]; then exit $rc; fi
for b in 160 192 224 256; do
  timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-c5 --batch $b 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, round(d['value']/1e10,3), round(d['pods_per_s']), d['kernels']['pods_per_launch'], round(d['kernels']['resolve_avg_ms']*1e3,1))" || exit 1
done
