# round-end evidence in one call: GPU tests, smoke, then bench + kernel trace + PMC passes (tools/gpu_profile_r01.sh)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
bash tools/gpu_profile_r01.sh
