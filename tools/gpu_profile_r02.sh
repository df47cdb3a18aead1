# Round-2 evidence: kernel-trace + stats of the collab bench (graph replay), dominant-launch trace summary
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o bench --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 > gpurun_out/prof_r02.log 2>&1
echo rc=$?
