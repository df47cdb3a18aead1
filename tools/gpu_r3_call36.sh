# per-kernel traces of the physics production step (BASELINE configs[3]): 1 rank and rank 0 of 4 (eager)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c36
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t1 -o t --output-format csv -- python tools/physics_bench.py --steps 10 --dtype bf16 > $O/t1.log 2>&1 || { tail $O/t1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t4 -o t --output-format csv -- python tools/physics_bench.py --steps 10 --dtype bf16 --emulate-ranks 4 > $O/t4.log 2>&1 || { tail $O/t4.log; exit 1; }
echo rc=0
