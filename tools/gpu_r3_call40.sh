# physics step: host time to enqueue a step vs the step time (eager and graph; 1 rank and rank 0 of 4)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c40
mkdir -p $O
for a in "" "--graph" "--emulate-ranks 4" "--emulate-ranks 4 --graph"; do
  timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 $a > $O/run.log 2>&1 || { tail $O/run.log; exit 1; }
  grep '^{"dtype' $O/run.log | head -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], round(d["ms_per_step"],4), round(d["host_issue_ms_per_step"],4))' "[$a]"
done
