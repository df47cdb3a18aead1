# segment-kernel tests under LLP_SEG_NPW=1/2/4, then a kernel trace of the collab step per setting
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 1 2 4; do
LLP_SEG_NPW=$n timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "segments" > gpurun_out/pytest_seg_$n.log 2>&1 || { echo tests failed $n; exit 1; }
done
T="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8"
for n in 1 2 4; do
LLP_SEG_NPW=$n timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_npw$n -o t --output-format csv -- $T > gpurun_out/trace_npw$n.log 2>&1 || exit 1
done
echo rc=$?
