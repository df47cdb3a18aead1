# A/B: non-temporal epilogue stores (LLP_GEMM_NT_STORE) on the collab step and the SAGE teacher step
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
B="python bench.py --no-eval --no-physics --no-cpu-baseline --steps 50"
for i in 1 2 3; do for v in 0 1; do
LLP_GEMM_NT_STORE=$v timeout -k 10 300 $B > gpurun_out/nts_b${v}_$i.json 2>&1 || exit 1
done; done
echo rc=$?
