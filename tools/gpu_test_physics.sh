export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_physics_fullsize.py tests/test_gpu_fullbatch.py tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > gpurun_out/it_pytest.log 2>&1
echo rc=$?
