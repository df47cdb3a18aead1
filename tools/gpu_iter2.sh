# Iteration: kernel + engine + teacher tests, teacher bench, student bench.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py tests/test_gpu_teacher.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it_pytest.log 2>&1 && \
timeout -k 10 300 python tools/sage_bench.py --dtype bf16 > gpurun_out/sage_bf16.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --no-sage > gpurun_out/it_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --emulate-ranks 8 --no-cpu-baseline --no-eval --no-sage > gpurun_out/it_r8.log 2>&1
echo rc=$?
