# per-call constant of the NT GEMM with and without the epilogue's stores / the whole epilogue
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
export LLP_AB_VARIANTS=${VARIANTS:-6,8}
timeout -k 10 200 python tools/gemm_k_sweep.py > gpurun_out/ks_full.log 2>&1 && \
LLP_LIB=$GRAFT_REPO_ROOT/tools/bin/NOSTORE/libllp_hip.so timeout -k 10 200 python tools/gemm_k_sweep.py > gpurun_out/ks_nostore.log 2>&1 && \
LLP_LIB=$GRAFT_REPO_ROOT/tools/bin/NOEPI/libllp_hip.so timeout -k 10 200 python tools/gemm_k_sweep.py > gpurun_out/ks_noepi.log 2>&1
echo rc=$?
