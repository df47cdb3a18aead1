# kernel trace of rank 0's shard of the collab step at 8 ranks (bench.py --emulate-ranks 8, hipGraph replay)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c38
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t8 -o t --output-format csv -- python bench.py --steps 10 --warmup 3 --emulate-ranks 8 > $O/t8.log 2>&1 || { tail $O/t8.log; exit 1; }
tail -2 $O/t8.log
