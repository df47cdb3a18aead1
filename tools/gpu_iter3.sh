# Iteration: teacher + kernel tests, teacher bench (bf16 / fp32).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_kernels.py tests/test_gpu_engine.py tests/test_gpu_fullbatch.py tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it_pytest.log 2>&1 && \
timeout -k 10 300 python tools/sage_bench.py --dtype bf16 > gpurun_out/sage_bf16.log 2>&1 && \
timeout -k 10 300 python tools/sage_bench.py --dtype fp32 > gpurun_out/sage_fp32.log 2>&1
echo rc=$?
