# Iteration check: targeted GPU tests, then bench variants (eager / graph / emulated 8 ranks).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
TESTS=${TESTS:-"tests/test_gpu_kernels.py tests/test_gpu_engine.py"}
timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/it_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py --no-graph --no-cpu-baseline --no-eval --no-sage > gpurun_out/it_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --graph --no-cpu-baseline --no-eval --no-sage > gpurun_out/it_bench_graph.log 2>&1 && \
timeout -k 10 300 python bench.py --emulate-ranks 8 --no-graph --no-cpu-baseline --no-eval --no-sage > gpurun_out/it_r8.log 2>&1 && \
timeout -k 10 300 python bench.py --emulate-ranks 8 --graph --no-cpu-baseline --no-eval --no-sage > gpurun_out/it_r8_graph.log 2>&1
echo rc=$?
