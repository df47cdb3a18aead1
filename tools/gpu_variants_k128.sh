# NT variants pp8-mode (11) vs h128 (5) on the collab shapes incl. the K=128 first student layer
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LLP_AB_VARIANTS=11,5 timeout -k 10 400 python tools/gemm_variants.py --rounds 3 > gpurun_out/variants_k128.log 2>&1
echo rc=$?
