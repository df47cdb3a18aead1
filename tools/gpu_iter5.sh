export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_citeseer_parity.py tests/test_gpu_cli.py -x -q --timeout 200 --timeout-method thread > gpurun_out/it_pytest.log 2>&1 && \
timeout -k 10 400 python tools/physics_bench.py --steps 10 --dtype bf16 > gpurun_out/physics.log 2>&1
echo rc=$?
