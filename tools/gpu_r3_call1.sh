# Round 3, first GPU call (gpurun --timeout 1500). Stops at the first failure.
#  1. the whole GPU suite (new dedup default: own scan + zeroing kernel, no rocprim / memset node)
#  2. segmented capture at the collab size, one rank, with a synchronising cut per stage,
#     replays checked bit for bit against eager steps (tools/seg_diag.py)
#  3. the same with two gloo ranks on the GPU (the configuration that faulted in round 2)
#  4. dedup passes traced for the default build, the wave segment sort and rocprim's scan
#  5. the gated tests of the round-2 opt-in paths (fp32 H=2048, head epilogue, sharded full batch)
#  6. last, as it may fault: the segmented capture with rocprim's scan and the zeroing kernel
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PYT tests -m gpu -q > gpurun_out/c1_pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 gpurun_out/c1_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/c1_pytest_gpu.log
timeout -k 10 300 python -u tools/seg_diag.py --debug-cuts > gpurun_out/c1_seg1.log 2>&1 || { echo "seg_diag 1 rank failed"; tail -30 gpurun_out/c1_seg1.log; exit 1; }
tail -1 gpurun_out/c1_seg1.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 tools/seg_diag.py > gpurun_out/c1_seg2.log 2>&1 || { echo "seg_diag 2 ranks failed"; tail -40 gpurun_out/c1_seg2.log; exit 1; }
grep '"rank"' gpurun_out/c1_seg2.log
for v in default wave rz; do
  if [ $v = default ]; then L=""; else L="LLP_LIB=tools/bin/libllp_hip_$v.so"; fi
  env $L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c1_dedup_$v -o t --output-format csv -- python tools/dedup_probe.py > gpurun_out/c1_dedup_$v.log 2>&1 || { echo "dedup probe $v failed"; exit 1; }
  tail -2 gpurun_out/c1_dedup_$v.log
done
LLP_TEST_WIDE=1 LLP_TEST_HEAD_LEAN=1 LLP_TEST_FB_SHARD=1 timeout -k 10 400 $PYT tests -m gpu -k "hidden_2048 or head_lean or fb_shard or segsort_wave" > gpurun_out/c1_gated.log 2>&1 || { echo "gated tests failed"; tail -40 gpurun_out/c1_gated.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED|passed|failed" gpurun_out/c1_gated.log | tail -15
LLP_LIB=tools/bin/libllp_hip_rz.so timeout -k 10 300 python -u tools/seg_diag.py --debug-cuts > gpurun_out/c1_seg1_rz.log 2>&1 || { echo "seg_diag rocprim scan failed"; tail -30 gpurun_out/c1_seg1_rz.log; exit 1; }
tail -1 gpurun_out/c1_seg1_rz.log
echo rc=0
