# First GPU call of the next round (one box, ~15 min; gpurun --timeout 1200): the whole GPU suite on the
# current tree, the opt-in head epilogue's gated test + kernel traces + step A/B, the
# node-sharded full-batch student's gated test + emulated 4-rank cost, the dedup's
# wave-per-segment sort (gated test + traces).  Stops at the first failure.  The
# segmented-capture bisection (tools/gpu_seg_bisect.sh, whose steps may fault) is the
# second call, on its own.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r3.log 2>&1 || { echo "gpu suite failed"; exit 1; }
echo "gpu suite: ok"
LLP_TEST_WIDE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v -m gpu --timeout 200 --timeout-method thread -k "hidden_2048" > gpurun_out/pytest_wide.log 2>&1 || { echo "wide fp32 test failed"; exit 1; }
echo "wide fp32 rows: ok"
bash tools/gpu_head_lean.sh || { echo "head epilogue A/B failed"; exit 1; }
echo "head epilogue A/B: done"
bash tools/gpu_fb_shard.sh || { echo "sharded full-batch student failed"; exit 1; }
echo "sharded full-batch student: done"
bash tools/gpu_segsort_wave.sh || { echo "segsort wave failed"; exit 1; }
echo "segsort wave: done"
echo rc=0
