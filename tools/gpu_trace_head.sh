# kernel trace of the collab step (graph replay) at HEAD, for per-kernel time and inter-kernel gaps
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_head -o t --output-format csv -- $B > gpurun_out/trace_head.log 2>&1
echo rc=$?
