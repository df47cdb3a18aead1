# TN stagger A/B (LLP_TN_STAG 0/1/2): GEMM micro-bench (TN rows) + collab step
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for i in 1 2; do for v in 0 1 2; do
LLP_TN_STAG=$v timeout -k 10 300 python tools/gemm_bench.py --iters 10 > gpurun_out/tns_g${v}_$i.txt 2>&1 || exit 1
LLP_TN_STAG=$v timeout -k 10 300 python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --steps 40 > gpurun_out/tns_b${v}_$i.json 2>&1 || exit 1
done; done
echo rc=$?
