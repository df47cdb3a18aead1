# Teacher (SAGE) step kernel breakdown + aggregate bandwidth, bf16 and fp32.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/sage_bench.py --dtype bf16 > gpurun_out/sage_bf16.log 2>&1 && \
timeout -k 10 300 python tools/sage_bench.py --dtype fp32 > gpurun_out/sage_fp32.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sage -o sage --output-format csv -- python tools/sage_bench.py --dtype bf16 --iters 5 --steps 5 > gpurun_out/prof_sage.log 2>&1
echo rc=$?
