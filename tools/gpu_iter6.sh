export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_teacher.py tests/test_gpu_cli.py -x -q --timeout 200 --timeout-method thread > gpurun_out/it_pytest.log 2>&1 && \
timeout -k 10 300 python tools/sage_bench.py --dtype bf16 > gpurun_out/sage_bf16.log 2>&1
echo rc=$?
