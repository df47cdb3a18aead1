# segment-kernel tests, then the collab step A/B: LLP_SEG_WAVE=0 (old) vs 1 (new), + per-kernel traces
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/ab_*.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q -m gpu --timeout 120 --timeout-method thread -k "segments or unique" > gpurun_out/pytest_seg.log 2>&1 || { echo tests failed; exit 1; }
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --no-shard8 --steps 50"
for i in 1 2 3; do
LLP_SEG_WAVE=0 timeout -k 10 300 $B > gpurun_out/ab_old_$i.json 2>&1 || exit 1
LLP_SEG_WAVE=1 timeout -k 10 300 $B > gpurun_out/ab_new_$i.json 2>&1 || exit 1
done
T="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8"
LLP_SEG_WAVE=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_a -o t --output-format csv -- $T > gpurun_out/trace_a.log 2>&1 || exit 1
LLP_SEG_WAVE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_b -o t --output-format csv -- $T > gpurun_out/trace_b.log 2>&1 || exit 1
echo rc=$?
