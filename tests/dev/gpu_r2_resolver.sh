# dev: the speculative resolver (KS_RESOLVER=2, the default) against the parity suite, then an
# A/B of both resolvers on the C3 bench (short, no CPU baseline, no C5 leg)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_engine_gpu.py tests/test_usage_keys_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r2b.log 2>&1
rc=$?; echo "small suite rc=$rc"; tail -4 gpurun_out/t_r2b.log; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do
  KS_RESOLVER=$R $T 200 python -u bench.py --steps 10 --no-cpu-baseline --no-c5 > gpurun_out/b_r2b_$R.json 2> gpurun_out/b_r2b_$R.log
  echo "bench resolver $R rc=$?"
  python3 -c "import json;d=json.load(open('gpurun_out/b_r2b_$R.json'));print(d['pods_per_s'], d['kernels'], d['roofline']['resolve'])"
done
$T 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/t_r2c.log 2>&1
rc=$?; echo "full suite rc=$rc"; tail -4 gpurun_out/t_r2c.log
