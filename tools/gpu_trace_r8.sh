# kernel trace of rank 0's shard of an 8-rank collab step (graph replay, no collective)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --emulate-ranks 8"
timeout -k 10 200 $B > gpurun_out/r8_plain.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_r8 -o t --output-format csv -- $B > gpurun_out/trace_r8.log 2>&1
echo rc=$?
