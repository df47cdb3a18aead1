# full-batch step with the dense negatives' count on the device + hipGraph replay: tests, physics graph vs eager;
# then the colsum / tile-walk A/Bs (call 26)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c27
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "fullbatch or physics or citeseer or train_parity or teacher or cli" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --no-graph > $O/p1_eager_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 > $O/p1_graph_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --emulate-ranks 4 --no-graph > $O/p4_eager_$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --emulate-ranks 4 > $O/p4_graph_$i.log 2>&1 || exit 1
done
for f in $O/p*_*.log; do echo "$f $(grep '^{"dtype' $f | head -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d.get("loss"), d.get("hipgraph"))')"; done
bash tools/gpu_r3_call26.sh
