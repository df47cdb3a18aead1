# lean NT epilogue A/B (tools/nt_epi_ab.py under each env; checksums must agree), then the GEMM kernel tests
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/epi_*.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "gemm or mask" > gpurun_out/pytest_epi.log 2>&1 || { echo tests failed; exit 1; }
for r in 1 2; do
for cfg in ${EPI_CFGS:-"LLP_GEMM_LEAN_EPI=0" "LLP_GEMM_LEAN_EPI=1"}; do
env $cfg timeout -k 10 200 python tools/nt_epi_ab.py >> gpurun_out/epi_ab.json 2> gpurun_out/epi_err.log || exit 1
done
done
echo rc=$?
