# Kernel breakdown of one rank's shard at R=8 (bench.py --emulate-ranks 8), N=1 for comparison.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r8 -o r8 --output-format csv -- python bench.py --steps 10 --warmup 3 --emulate-ranks 8 --no-cpu-baseline --no-eval --no-sage --no-physics > gpurun_out/prof_r8.log 2>&1
echo rc=$?
