# World-size-2 RCCL rehearsal of the C5 node-sharded path on a one-GPU box (both ranks on the same
# device; functional only — the numbers mean nothing).  Compared with the unsharded N=1 binds by
# the C5 test suite; here it must simply complete and report.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
KS_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --config c5 --gpus 2 --steps 2 --warmup 1 --c5-pods 70000 > gpurun_out/c5_n2.json 2> gpurun_out/c5_n2.log
rc=$?
echo "rc=$rc"
tail -5 gpurun_out/c5_n2.log
cat gpurun_out/c5_n2.json | cut -c1-300
