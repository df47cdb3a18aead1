# Hadamard-rows tests, then kernel traces of the collab step with LLP_HADA_WAVE=0 / 1
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "hadamard" > gpurun_out/pytest_hada.log 2>&1 || { echo tests failed; exit 1; }
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8"
LLP_HADA_WAVE=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_a -o t --output-format csv -- $B > gpurun_out/trace_a.log 2>&1 || exit 1
LLP_HADA_WAVE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_b -o t --output-format csv -- $B > gpurun_out/trace_b.log 2>&1 || exit 1
echo rc=$?
