# physics step, rank 0 of 4: kernel trace of the hipGraph replay (capture_fullbatch) beside the eager one (call 36)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c39
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/g4 -o t --output-format csv -- python tools/physics_bench.py --steps 10 --dtype bf16 --emulate-ranks 4 --graph > $O/g4.log 2>&1 || { tail $O/g4.log; exit 1; }
grep '^{"dtype' $O/g4.log | head -2
