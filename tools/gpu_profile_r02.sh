# Round-2 evidence: default bench line, kernel-trace + stats of the collab step (graph replay),
# FETCH_SIZE / WRITE_SIZE passes of the dominant GEMM (bench --dominant-only)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > gpurun_out/bench_r02.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o bench --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 > gpurun_out/prof_r02.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_r02 -o run --output-format csv -- python bench.py --dominant-only 10 --no-cpu-baseline --no-eval --no-sage > gpurun_out/pmc_fetch_r02.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_r02 -o run --output-format csv -- python bench.py --dominant-only 10 --no-cpu-baseline --no-eval --no-sage > gpurun_out/pmc_write_r02.log 2>&1
echo rc=$?
