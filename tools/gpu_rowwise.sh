# per-rank cost table: unique-node vs row-wise student (LLP_DEDUP=0), whole batch and rank 0's 8-rank shard
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --steps 30"
timeout -k 10 300 $B > gpurun_out/rw_dedup.json 2>&1 && \
LLP_DEDUP=0 timeout -k 10 300 $B > gpurun_out/rw_rowwise.json 2>&1
echo rc=$?
