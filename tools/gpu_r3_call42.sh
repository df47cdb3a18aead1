# Adam blocks of 1024 elements (default) vs 4096 (adam4096): optimizer tests, physics (1 / 4 ranks) and collab steps
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c42
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "adam or optim or clip or engine or fullbatch or golden or train_parity" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L="new=linkless-link-prediction_amd/libllp_hip.so old=tools/bin/libllp_hip_adam4096.so"
timeout -k 10 400 python -u tools/ab_gemm.py $L --rounds 3 --script tools/physics_bench.py --args "--steps 20 --dtype bf16" > $O/ab_p1.log 2>&1 || { tail -20 $O/ab_p1.log; exit 1; }
tail -1 $O/ab_p1.log
timeout -k 10 400 python -u tools/ab_gemm.py $L --rounds 3 --script tools/physics_bench.py --args "--steps 20 --dtype bf16 --emulate-ranks 4 --graph" > $O/ab_p4.log 2>&1 || { tail -20 $O/ab_p4.log; exit 1; }
tail -1 $O/ab_p4.log
timeout -k 10 600 python -u tools/ab_gemm.py $L --rounds 3 --script bench.py --args "--steps 30 --warmup 5 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32 --no-practical-peak" > $O/ab_collab.log 2>&1 || { tail -20 $O/ab_collab.log; exit 1; }
tail -1 $O/ab_collab.log
