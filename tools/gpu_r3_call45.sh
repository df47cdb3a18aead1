# dense negatives: membership through the edge set (default) vs the sorted-key binary search (--no-edge-table):
# the kernel and engine tests, then the physics step at 1 rank and rank 0 of 4, 3 interleaved rounds
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c45
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "neg or fullbatch or physics or teacher or citeseer or train_parity or cli" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for v in new old; do
    F=""; [ $v = old ] && F="--no-edge-table"
    timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 $F > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
    timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --emulate-ranks 4 --graph $F > $O/p4.log 2>&1 || { tail $O/p4.log; exit 1; }
    echo "$v $r $(grep '^{"dtype' $O/p1.log | head -1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],4))') $(grep '^{"dtype' $O/p4.log | head -1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],4))')" | tee -a $O/ab.txt
  done
done
