# colsum/head tests, then the collab-step kernel trace (colsum_vec_kernel time) and a short bench
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "head or segments" > gpurun_out/pytest_colsum.log 2>&1 || { echo tests failed; exit 1; }
T="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_cs -o t --output-format csv -- $T > gpurun_out/trace_cs.log 2>&1 || exit 1
echo rc=$?
