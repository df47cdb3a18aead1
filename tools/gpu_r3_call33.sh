# head-backward colsum: 8 (default) vs 12 vs 16 rows in flight per lane, same box
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c33
mkdir -p $O
timeout -k 10 300 python -u tools/ab_gemm.py default=linkless-link-prediction_amd/libllp_hip.so nf12=tools/bin/libllp_hip_colsum12.so nf16=tools/bin/libllp_hip_colsum16.so --rounds 3 --script tools/colsum_bench.py > $O/ab_colsum.log 2>&1 || { tail -20 $O/ab_colsum.log; exit 1; }
tail -1 $O/ab_colsum.log
