# interleaved A/B of NT GEMM variants (LLP_AB_VARIANTS) on the collab shapes, bit-identity check first
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LLP_AB_VARIANTS=${VARIANTS:-6,8} timeout -k 10 300 python tools/gemm_variants.py --rounds ${ROUNDS:-5} > gpurun_out/variants.log 2>&1
echo rc=$?
