# full-batch step: student forward queued before the dense negatives' host read; physics A/B against the
# previous engine (a copy of the tree with tools/bin/llp_engine_prev.py), plus the GPU suite's full-batch tests
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c17
mkdir -p $O
OLD=/tmp/llp_old_tree
rm -rf $OLD && mkdir -p $OLD && cp -r linkless-link-prediction_amd tools oracle bench.py $OLD/ && cp tools/bin/llp_engine_prev.py $OLD/linkless-link-prediction_amd/llp_engine.py
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests -m gpu -k "fullbatch or physics or fb_shard or train_parity or golden" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  (cd $OLD && timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --emulate-ranks 4) > $O/p4_old_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --emulate-ranks 4 > $O/p4_new_$i.log 2>&1 || exit 1
  (cd $OLD && timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16) > $O/p1_old_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 > $O/p1_new_$i.log 2>&1 || exit 1
done
for f in $O/p*_*.log; do echo "$f $(grep '^{' $f | head -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d.get("loss"))')"; done
echo rc=0
