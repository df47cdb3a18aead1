# kernel-trace summary of the coauthor-physics production step: whole batch, and rank 0's shard at 4 ranks
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_phys1 -o p1 --output-format csv -- python tools/physics_bench.py --steps 10 > gpurun_out/prof_phys1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_phys4 -o p4 --output-format csv -- python tools/physics_bench.py --steps 10 --emulate-ranks 4 > gpurun_out/prof_phys4.log 2>&1
echo rc=$?
