export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_parity.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/it_pytest.log 2>&1
echo rc=$?
