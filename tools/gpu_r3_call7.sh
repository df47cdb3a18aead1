# bf16 accuracy test; per-kernel traces of rank 0's shard at 8 ranks and of the whole step (collab)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread tests/test_gpu_bf16_accuracy.py > gpurun_out/c7_acc.log 2>&1 || { echo "accuracy test failed"; tail -30 gpurun_out/c7_acc.log; exit 1; }
grep -E "passed|failed" gpurun_out/c7_acc.log | tail -1
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c7_trace_r8 -o run --output-format csv -- $B --emulate-ranks 8 > gpurun_out/c7_trace_r8.log 2>&1 || { echo "trace r8 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c7_trace_r1 -o run --output-format csv -- $B --emulate-ranks 1 > gpurun_out/c7_trace_r1.log 2>&1 || { echo "trace r1 failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32 --emulate-ranks 8 > gpurun_out/c7_r8.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32 --emulate-ranks 1 > gpurun_out/c7_r1.json 2>&1 || exit 1
tail -qn1 gpurun_out/c7_r8.json gpurun_out/c7_r1.json
echo rc=0
