# optimizer-tail changes: kernel + engine + golden-replay GPU tests, then the step and the 8-rank shard
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
for i in 1 2; do timeout -k 10 300 python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --steps 50 > gpurun_out/adam_$i.json 2>&1 || exit 1; done
echo rc=$?
