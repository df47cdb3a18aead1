# second-stream overlap modes (LLP_OVERLAP) on rank 0's 8-rank shard (eager, so the side stream is live)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for i in 1 2; do for m in 0 1 2 4 7; do
LLP_OVERLAP=$m timeout -k 10 300 python bench.py --emulate-ranks 8 --steps 40 --no-graph > gpurun_out/ovr8_${m}_$i.json 2>&1 || exit 1
done; done
echo rc=$?
