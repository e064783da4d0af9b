# dev: speculative resolver A/B + per-wave stamps (short runs)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_engine_gpu.py tests/test_usage_keys_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r2d.log 2>&1
rc=$?; echo "small suite rc=$rc"; tail -4 gpurun_out/t_r2d.log; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do
  KS_RESOLVER=$R $T 200 python -u bench.py --steps 10 --no-cpu-baseline --no-c5 > gpurun_out/b_r2d_$R.json 2> gpurun_out/b_r2d_$R.log
  echo "bench resolver $R rc=$?"
  python3 -c "import json;d=json.load(open('gpurun_out/b_r2d_$R.json'));print(d['pods_per_s'], d['kernels'], d['roofline']['resolve']['ns_per_pod'])"
done
$T 200 python -u tests/dev/diag_resolve2.py 256
KS_RESOLVER=2 timeout -k 10 200 python -u bench.py --config c4 --steps 2 --warmup 1 > gpurun_out/b_r2d_c4.json 2> gpurun_out/b_r2d_c4.log; echo "c4 rc=$?"; cat gpurun_out/b_r2d_c4.json | head -c 600
