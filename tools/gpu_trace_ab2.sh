# kernel traces of the collab step under ENV_A / ENV_B (per-kernel A/B with tools/trace_step.py)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 ${BENCH_EXTRA}"
env $ENV_A timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_a -o t --output-format csv -- $B > gpurun_out/trace_a.log 2>&1 || exit 1
env $ENV_B timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_b -o t --output-format csv -- $B > gpurun_out/trace_b.log 2>&1 || exit 1
echo rc=$?
