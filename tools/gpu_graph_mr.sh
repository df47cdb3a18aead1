# multi-rank hipGraph segments: the 2-rank gloo tests, then bench.py at N=2 rehearsed on one GPU (gloo)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_mr.log 2>&1 || exit 1
LLP_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-eval --no-sage > gpurun_out/bench_n2_gloo.log 2>&1 || exit 1
LLP_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --no-eval --no-sage --no-graph > gpurun_out/bench_n2_gloo_eager.log 2>&1
echo rc=$?
