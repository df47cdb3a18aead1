# persistent NT epilogue with balanced conversion rounds: bit-identity tests, then A/B against the previous build
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c23
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu -k "persistent or lean or head" > $O/kt.log 2>&1 || { tail -30 $O/kt.log; exit 1; }
tail -1 $O/kt.log
timeout -k 10 400 python tools/ab_gemm.py old=tools/bin/libllp_hip_old.so new=tools/bin/libllp_hip_new.so --rounds 3 > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
tail -1 $O/ab.log
echo rc=0
