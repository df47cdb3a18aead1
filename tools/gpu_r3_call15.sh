# memory-bound kernels of the collab step with the current build: PMC FETCH / WRITE passes + kernel trace
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c15
mkdir -p $O
S="python bench.py --no-graph --steps 4 --warmup 2 --profile-kernels --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $S > $O/pmc_fetch.log 2>&1 || { tail $O/pmc_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $S > $O/pmc_write.log 2>&1 || { tail $O/pmc_write.log; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- $S > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
echo rc=0
