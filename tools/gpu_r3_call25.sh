# contiguous-range tile walk of the persistent NT GEMM: bit-identity tests on that build, then A/B
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c25
mkdir -p $O
LLP_LIB=tools/bin/libllp_hip_walk.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "persistent" > $O/kt.log 2>&1 || { tail -30 $O/kt.log; exit 1; }
tail -1 $O/kt.log
timeout -k 10 400 python tools/ab_gemm.py default=linkless-link-prediction_amd/libllp_hip.so walk=tools/bin/libllp_hip_walk.so --rounds 3 > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
tail -1 $O/ab.log
echo rc=0
