export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o bench --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 > gpurun_out/prof_r01.log 2>&1
echo rc=$?
