# GPU tests + the collab bench (no side legs) + the 8-rank emulated shard
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --steps 30 > gpurun_out/quick_bench.json 2>&1 && \
timeout -k 10 300 python bench.py --emulate-ranks 8 --steps 30 > gpurun_out/quick_r8.json 2>&1
echo rc=$?
