# GPU tests (all), then the collab step A/B LLP_GEMM_LEAN_EPI=0 vs 1 (3 interleaved rounds of 50 steps)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/ab_*.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo tests failed; exit 1; }
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --no-shard8 --steps 50"
for i in 1 2 3; do
LLP_GEMM_LEAN_EPI=0 timeout -k 10 300 $B > gpurun_out/ab_old_$i.json 2>&1 || exit 1
LLP_GEMM_LEAN_EPI=1 timeout -k 10 300 $B > gpurun_out/ab_new_$i.json 2>&1 || exit 1
done
echo rc=$?
