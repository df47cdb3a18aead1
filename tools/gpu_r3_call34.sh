# empty-input C-ABI tests and the wider rw_step sampler cases first, then the whole GPU suite
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c34
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_empty.py tests/test_gpu_kernels.py -k "empty or zero or sampler or isolated or no_negatives" > $O/pytest_new.log 2>&1 || { echo "new tests failed"; tail -40 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
