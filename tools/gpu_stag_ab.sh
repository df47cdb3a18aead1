# staggered q64 variants: bit-identity + interleaved micro A/B, then the collab bench per variant
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/gemm_variants.py --rounds 5 --iters 10 > gpurun_out/stag_variants.txt 2>&1 || exit 1
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --steps 30"
for i in 1 2; do for v in 4 6 7; do
timeout -k 10 300 env LLP_GEMM_VARIANT=$v $B > gpurun_out/stag_b${v}_$i.json 2> gpurun_out/stag_b${v}_$i.err || exit 1
done; done
echo rc=$?
