# GEMM workgroup stamps (diagnostic build); wave-per-anchor Hadamard anchor sums vs thread-per-chunk (A/B traces)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "segments or hadamard or dedup or unique" > gpurun_out/c8_pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c8_pytest.log; exit 1; }
tail -1 gpurun_out/c8_pytest.log
timeout -k 10 200 python -u tools/gemm_stamps.py > gpurun_out/c8_stamps.json 2> gpurun_out/c8_stamps.err || { echo "stamps failed"; tail -20 gpurun_out/c8_stamps.err; exit 1; }
cat gpurun_out/c8_stamps.json
T="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32"
for i in 1 2; do
LLP_LIB=tools/bin/libllp_hip_anchor_threads.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c8_tr_thr$i -o t --output-format csv -- $T > gpurun_out/c8_tr_thr$i.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c8_tr_wave$i -o t --output-format csv -- $T > gpurun_out/c8_tr_wave$i.log 2>&1 || exit 1
done
python tools/trace_summary.py gpurun_out/c8_tr_thr1 gpurun_out/c8_tr_wave1 gpurun_out/c8_tr_thr2 gpurun_out/c8_tr_wave2 -k anchor segments_wave > gpurun_out/c8_anchor_ab.txt || exit 1
cat gpurun_out/c8_anchor_ab.txt
echo rc=0
