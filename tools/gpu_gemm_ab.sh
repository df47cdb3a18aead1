# NT GEMM variant A/B (q64-lean vs h128) at the step's shapes, then the gemm kernel tests under h128.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/gemm_variants.py --rounds 5 --iters 10 > gpurun_out/gemm_ab.log 2>&1 && \
LLP_GEMM_VARIANT=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/it_pytest_h128.log 2>&1
echo rc=$?
