# rehearsal of the N=2 bench path on one GPU (2 ranks share the device, gloo)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LLP_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-sage --no-physics > gpurun_out/bench2_gloo.log 2>&1
echo rc=$?
