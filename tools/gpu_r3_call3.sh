# Round 3, third GPU call (gpurun --timeout 1500).  Stops at the first failure.
#  1. the whole GPU suite
#  2. PMC FETCH / WRITE passes + kernel trace of eager collab steps (memory-bound kernels)
#  3. SAGE aggregate: every configuration, PMC passes (rows-per-wave kernel) and the
#     event-timed A/B against the lane-group kernel (tools/bin/libllp_hip_agg_groups.so)
#  4. the default bench line
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $PYT tests -m gpu -q > gpurun_out/c3_pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/c3_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/c3_pytest_gpu.log
S="python bench.py --no-graph --steps 4 --warmup 2 --profile-kernels --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c3_pmc_step_fetch -o run --output-format csv -- $S > gpurun_out/c3_pmc_step_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c3_pmc_step_write -o run --output-format csv -- $S > gpurun_out/c3_pmc_step_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c3_trace_step -o run --output-format csv -- $S > gpurun_out/c3_trace_step.log 2>&1 || { echo "trace failed"; exit 1; }
A="python tools/sage_bench.py --agg-only --iters 10"
timeout -k 10 180 $A > gpurun_out/c3_sage_plan.json 2> gpurun_out/c3_sage_plan.err || { echo "sage plan failed"; tail gpurun_out/c3_sage_plan.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c3_pmc_sage_fetch -o run --output-format csv -- $A > gpurun_out/c3_pmc_sage_fetch.log 2>&1 || { echo "sage pmc fetch failed"; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c3_pmc_sage_write -o run --output-format csv -- $A > gpurun_out/c3_pmc_sage_write.log 2>&1 || { echo "sage pmc write failed"; exit 1; }
for i in 1 2; do
LLP_LIB=tools/bin/libllp_hip_agg_groups.so timeout -k 10 180 $A --iters 30 > gpurun_out/c3_sage_groups_$i.json 2>/dev/null || exit 1
timeout -k 10 180 $A --iters 30 > gpurun_out/c3_sage_rows_$i.json 2>/dev/null || exit 1
done
timeout -k 10 600 python bench.py > gpurun_out/c3_bench1.json 2> gpurun_out/c3_bench1.err || { echo "bench N=1 failed"; tail -20 gpurun_out/c3_bench1.err; exit 1; }
echo rc=0
