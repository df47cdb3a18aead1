# whole GPU suite, the default bench line, and a kernel-trace + stats profile of the bench (round-3 final profiles)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c28
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 300 $O/bench.json
T="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o t --output-format csv -- $T > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
echo rc=0
