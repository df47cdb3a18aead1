# is the NT main loop waiting on A-operand fetches?  default and no-epilogue builds with A rows
# aliased to one row (always an L2 hit) against real A rows
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c24
mkdir -p $O
timeout -k 10 300 python tools/ab_gemm.py default=linkless-link-prediction_amd/libllp_hip.so skip=tools/bin/libllp_hip_epi_skip.so --rounds 2 > $O/real.log 2>&1 || { tail $O/real.log; exit 1; }
tail -1 $O/real.log
timeout -k 10 300 python tools/ab_gemm.py default=linkless-link-prediction_amd/libllp_hip.so skip=tools/bin/libllp_hip_epi_skip.so --rounds 2 --a-one-row > $O/onerow.log 2>&1 || { tail $O/onerow.log; exit 1; }
tail -1 $O/onerow.log
echo rc=0
