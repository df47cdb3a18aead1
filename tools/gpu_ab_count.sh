# Same-box A/B: device-resident unique count (default) vs host read (LLP_DEVICE_COUNT=0), twice each.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it_pytest.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --no-sage > gpurun_out/ab_dev_$i.log 2>&1 && \
LLP_DEVICE_COUNT=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-eval --no-sage > gpurun_out/ab_host_$i.log 2>&1 || exit 1
done
echo rc=$?
