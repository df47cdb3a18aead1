# Opt-in wave-per-segment sort of the dedup (LLP_SEGSORT=wave): its gated
# kernel test, then kernel traces of the stress probe and of the step's own targets, default
# vs wave (same outputs: the probes print checksums).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LLP_TEST_SEGSORT_WAVE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu --timeout 120 --timeout-method thread -k "segsort_wave or dedup_rows" > gpurun_out/pytest_segsort_wave.log 2>&1 || { echo tests failed; exit 1; }
for v in default wave; do
if [ $v = wave ]; then export LLP_SEGSORT=wave; fi
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/ssw_probe_$v -o t --output-format csv -- python tools/dedup_probe.py > gpurun_out/ssw_probe_$v.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ssw_step_$v -o t --output-format csv -- python tools/dedup_step_probe.py --ranks 1 > gpurun_out/ssw_step_$v.log 2>&1 || exit 1
done
python tools/trace_summary.py gpurun_out/ssw_probe_default gpurun_out/ssw_probe_wave gpurun_out/ssw_step_default gpurun_out/ssw_step_wave -k segsort > gpurun_out/segsort_wave.txt || exit 1
echo rc=0
