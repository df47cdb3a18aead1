# GPU tests + smoke + variant A/B (bit identity) + bench
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
LLP_AB_VARIANTS=${VARIANTS:-6,11} timeout -k 10 300 python tools/gemm_variants.py --rounds 3 > gpurun_out/variants.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1
echo rc=$?
