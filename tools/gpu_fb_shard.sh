# Opt-in node-sharded full-batch student (LLP_FB_SHARD): the engine's gated
# 2-rank gloo test on the one GPU, then rank 0's per-step cost at 4 ranks of the
# coauthor-physics production step, replicated vs sharded student (emulated, no collective).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LLP_TEST_FB_SHARD=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -x -v -m gpu --timeout 300 --timeout-method thread -k "fullbatch" > gpurun_out/pytest_fb_shard.log 2>&1 || { echo tests failed; exit 1; }
timeout -k 10 300 python tools/physics_bench.py --dtype bf16 --emulate-ranks 4 > gpurun_out/physics_r4_repl.log 2>&1 || exit 1
LLP_FB_SHARD=1 timeout -k 10 300 python tools/physics_bench.py --dtype bf16 --emulate-ranks 4 > gpurun_out/physics_r4_shard.log 2>&1 || exit 1
echo rc=0
