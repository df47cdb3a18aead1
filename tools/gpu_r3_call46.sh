# whole GPU suite and the default bench line (round-3 closing check of the committed tree)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c46
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
echo rc=0
