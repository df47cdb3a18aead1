# multi-rank GPU tests with the 4-rank cases (4 gloo ranks on one GPU)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c35
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_multirank.py > $O/pytest_multirank.log 2>&1 || { echo "multirank failed"; tail -40 $O/pytest_multirank.log; exit 1; }
tail -3 $O/pytest_multirank.log
