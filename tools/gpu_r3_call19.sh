# norm_type 'layer' / 'batch': the norm kernel / module / engine tests, the golden replays with norms, then the whole GPU suite
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c19
mkdir -p $O
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_norm.py -m gpu > $O/norm.log 2>&1 || { echo "norm tests failed"; grep -E "PASS|FAIL|Error|assert" $O/norm.log | tail -40; exit 1; }
grep -c PASSED $O/norm.log
timeout -k 10 600 $PYT tests -m gpu -k "norm" > $O/norm_all.log 2>&1 || { echo "norm replays failed"; grep -E "PASS|FAIL|Error|assert" $O/norm_all.log | tail -40; exit 1; }
grep -c PASSED $O/norm_all.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
echo rc=0
