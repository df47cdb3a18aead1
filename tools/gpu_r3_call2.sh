# Round 3, second GPU call (gpurun --timeout 1500).  Stops at the first failure.
#  1. hipMemsetAsync node under the segmented capture (fault-free probe with guard words)
#  2. the whole GPU suite (wave segment sort default, un-gated fp32 H=2048, collab-node segmented graph)
#  3. fb-shard gated 2-rank test + rank 0's emulated 4-rank physics step, replicated vs sharded
#  4. head-lean epilogue: kernel traces + 3 interleaved step A/B rounds
#  5. bench N=1 (default line) and N=2 gloo rehearsal with the segmented graph
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $PYT tests -m gpu -q > gpurun_out/c2_pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/c2_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/c2_pytest_gpu.log
LLP_TEST_FB_SHARD=1 timeout -k 10 400 $PYT tests/test_gpu_multirank.py -m gpu -k "sharded_student" > gpurun_out/c2_fb_shard.log 2>&1 || { echo "fb shard test failed"; tail -30 gpurun_out/c2_fb_shard.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/c2_fb_shard.log | tail -3
for i in 1 2; do
timeout -k 10 300 python tools/physics_bench.py --dtype bf16 --emulate-ranks 4 > gpurun_out/c2_phys_repl_$i.log 2>&1 || exit 1
LLP_FB_SHARD=1 timeout -k 10 300 python tools/physics_bench.py --dtype bf16 --emulate-ranks 4 > gpurun_out/c2_phys_shard_$i.log 2>&1 || exit 1
done
tail -qn1 gpurun_out/c2_phys_*.log
T="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8"
for v in 0 1; do
LLP_GEMM_HEAD_LEAN=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c2_trace_hl$v -o t --output-format csv -- $T > gpurun_out/c2_trace_hl$v.log 2>&1 || exit 1
done
python tools/trace_summary.py gpurun_out/c2_trace_hl0 gpurun_out/c2_trace_hl1 -k "pp8" > gpurun_out/c2_head_lean_kernels.txt || exit 1
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --no-shard8 --steps 50"
for i in 1 2 3; do
LLP_GEMM_HEAD_LEAN=0 timeout -k 10 300 $B > gpurun_out/c2_hl_old_$i.json 2>&1 || exit 1
LLP_GEMM_HEAD_LEAN=1 timeout -k 10 300 $B > gpurun_out/c2_hl_new_$i.json 2>&1 || exit 1
done
timeout -k 10 600 python bench.py > gpurun_out/c2_bench1.json 2> gpurun_out/c2_bench1.err || { echo "bench N=1 failed"; tail -20 gpurun_out/c2_bench1.err; exit 1; }
LLP_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-sage --no-physics --no-eval > gpurun_out/c2_bench2_gloo.log 2>&1 || { echo "bench N=2 gloo failed"; tail -30 gpurun_out/c2_bench2_gloo.log; exit 1; }
grep '"metric"' gpurun_out/c2_bench2_gloo.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=2 gloo', d['ms_per_step'], d['hipgraph'])"
echo rc=0
