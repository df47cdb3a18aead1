export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --dominant-only 10 --no-cpu-baseline --no-eval --no-sage > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --dominant-only 10 --no-cpu-baseline --no-eval --no-sage > gpurun_out/pmc_write.log 2>&1
echo rc=$?
