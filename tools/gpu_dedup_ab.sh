# counting-sort compaction (default) vs the radix path (LLP_DEDUP_SORT=radix): kernel tests + collab step + 8-rank shard
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "dedup or segment" > gpurun_out/pytest_dedup.log 2>&1 || exit 1
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --steps 40"
for i in 1 2; do
timeout -k 10 300 $B > gpurun_out/dd_count_$i.json 2>&1 || exit 1
LLP_DEDUP_SORT=radix timeout -k 10 300 $B > gpurun_out/dd_radix_$i.json 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo rc=$?
