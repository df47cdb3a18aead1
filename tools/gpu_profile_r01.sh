# Round-1 evidence: bench line, kernel-trace summary, PMC passes of the dominant GEMM.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > gpurun_out/bench_r01.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01 -o bench --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 > gpurun_out/prof_r01.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --dominant-only 10 --no-cpu-baseline --no-eval --no-sage > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --dominant-only 10 --no-cpu-baseline --no-eval --no-sage > gpurun_out/pmc_write.log 2>&1
echo rc=$?
