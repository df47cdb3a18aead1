# re-entry check of HEAD: the whole GPU suite, the default bench line, physics step at 1 rank and rank 0 of 4
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c18
mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 > $O/p1.log 2>&1 || exit 1
timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --emulate-ranks 4 > $O/p4.log 2>&1 || exit 1
grep '^{' $O/p1.log $O/p4.log | cut -c1-300
echo rc=0
