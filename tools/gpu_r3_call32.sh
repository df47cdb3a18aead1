# NT epilogue pricing: default vs no C stores vs no epilogue vs stores aliased into L2 (tools/gemm_epi_cost.py)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c32
mkdir -p $O
timeout -k 10 400 python -u tools/gemm_epi_cost.py --rounds 3 > $O/epi_cost.log 2>&1 || { tail -20 $O/epi_cost.log; exit 1; }
tail -1 $O/epi_cost.log
