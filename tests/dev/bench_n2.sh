# N=2 rehearsal on a one-GPU box: two ranks share the GPU (C3 replicas; the C5 leg reports why it
# is skipped), the driver's launch line.
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/b_n2.json 2> gpurun_out/b_n2.log
rc=$?
echo "rc=$rc"
cat gpurun_out/b_n2.json | cut -c1-400
