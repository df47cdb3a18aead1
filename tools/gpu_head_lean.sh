# Opt-in lean head epilogue (LLP_GEMM_HEAD_LEAN): its gated kernel
# test, the head-mode GEMM per launch from kernel traces (0 / 1), then the collab step
# A/B in 3 interleaved rounds.  Stops at the first failure.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/hl_*.json
LLP_TEST_HEAD_LEAN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu --timeout 120 --timeout-method thread -k "head" > gpurun_out/pytest_head_lean.log 2>&1 || { echo tests failed; exit 1; }
T="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8"
for v in 0 1; do
LLP_GEMM_HEAD_LEAN=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_hl$v -o t --output-format csv -- $T > gpurun_out/trace_hl$v.log 2>&1 || exit 1
done
python tools/trace_summary.py gpurun_out/trace_hl0 gpurun_out/trace_hl1 -k "pp8" > gpurun_out/head_lean_kernels.txt || exit 1
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --no-shard8 --steps 50"
for i in 1 2 3; do
LLP_GEMM_HEAD_LEAN=0 timeout -k 10 300 $B > gpurun_out/hl_old_$i.json 2>&1 || exit 1
LLP_GEMM_HEAD_LEAN=1 timeout -k 10 300 $B > gpurun_out/hl_new_$i.json 2>&1 || exit 1
done
echo rc=0
