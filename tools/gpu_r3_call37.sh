# TN split count filling whole waves (default) vs the round-up (LLP_TN_SPLITS_CEIL): physics step at 1 rank and
# rank 0 of 4, then the GPU tests that run the TN GEMM
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c37
mkdir -p $O
L="new=linkless-link-prediction_amd/libllp_hip.so ceil=tools/bin/libllp_hip_tnceil.so"
timeout -k 10 400 python -u tools/ab_gemm.py $L --rounds 3 --script tools/physics_bench.py --args "--steps 20 --dtype bf16" > $O/ab_p1.log 2>&1 || { tail -20 $O/ab_p1.log; exit 1; }
tail -1 $O/ab_p1.log
timeout -k 10 400 python -u tools/ab_gemm.py $L --rounds 3 --script tools/physics_bench.py --args "--steps 20 --dtype bf16 --emulate-ranks 4" > $O/ab_p4.log 2>&1 || { tail -20 $O/ab_p4.log; exit 1; }
tail -1 $O/ab_p4.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
