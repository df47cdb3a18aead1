# split-K GEMM: kernel tests, the whole GPU suite, physics step A/B (1 rank, rank 0 of 4) against no split
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c16
mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_kernels.py -m gpu -k "splitk" > $O/splitk.log 2>&1 || { echo "splitk tests failed"; tail -30 $O/splitk.log; exit 1; }
tail -1 $O/splitk.log
timeout -k 10 900 $PYT tests -m gpu > $O/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
P="python tools/physics_bench.py --steps 20 --dtype bf16"
for i in 1 2; do
  LLP_LIB=tools/bin/libllp_hip_nosplitk.so timeout -k 10 300 $P > $O/p1_old_$i.log 2>&1 || exit 1
  timeout -k 10 300 $P > $O/p1_new_$i.log 2>&1 || exit 1
  LLP_LIB=tools/bin/libllp_hip_nosplitk.so timeout -k 10 300 $P --emulate-ranks 4 > $O/p4_old_$i.log 2>&1 || exit 1
  timeout -k 10 300 $P --emulate-ranks 4 > $O/p4_new_$i.log 2>&1 || exit 1
done
for f in $O/p*_*.log; do echo "$f $(grep '^{' $f | head -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d.get("loss"))')"; done
echo rc=0
