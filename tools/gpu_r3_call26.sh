# colsum with 8 rows in flight per lane (A/B against 4) and the contiguous-range GEMM tile walk (A/B)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c26
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fullbatch.py -m gpu -k "colsum or head" > $O/kt.log 2>&1 || { tail -30 $O/kt.log; exit 1; }
tail -1 $O/kt.log
timeout -k 10 300 python tools/ab_gemm.py in8=linkless-link-prediction_amd/libllp_hip.so in4=tools/bin/libllp_hip_colsum4.so --rounds 3 --script tools/colsum_bench.py > $O/colsum_ab.log 2>&1 || { tail $O/colsum_ab.log; exit 1; }
tail -1 $O/colsum_ab.log
LLP_LIB=tools/bin/libllp_hip_walk.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "persistent" > $O/kt_walk.log 2>&1 || { tail -30 $O/kt_walk.log; exit 1; }
tail -1 $O/kt_walk.log
timeout -k 10 400 python tools/ab_gemm.py default=linkless-link-prediction_amd/libllp_hip.so walk=tools/bin/libllp_hip_walk.so --rounds 3 > $O/walk_ab.log 2>&1 || { tail $O/walk_ab.log; exit 1; }
tail -1 $O/walk_ab.log
echo rc=0
