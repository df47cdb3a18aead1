# Per-rank cost at 8 ranks: kernel-trace summary of rank 0's shard (bench --emulate-ranks 8), graph and eager
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --emulate-ranks 8 --steps 30 > gpurun_out/r8_graph.json 2>&1 && \
timeout -k 10 300 python bench.py --emulate-ranks 8 --steps 30 --no-graph > gpurun_out/r8_eager.json 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r8 -o r8 --output-format csv -- python bench.py --emulate-ranks 8 --steps 10 --warmup 2 > gpurun_out/prof_r8.log 2>&1
echo rc=$?
