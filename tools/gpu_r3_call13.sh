# per-rank breakdowns for DESIGN §5: rank 0's shard of the collab step at 8 ranks, the physics
# full-batch step at 1 and 4 ranks (sharded student, and replicated), kernel traces + timelines
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c13
mkdir -p $O
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_r8 -o t --output-format csv -- $B --emulate-ranks 8 > $O/tr_r8.log 2>&1 || { tail $O/tr_r8.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_p1 -o t --output-format csv -- python tools/physics_bench.py --steps 10 > $O/tr_p1.log 2>&1 || { tail $O/tr_p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_p4 -o t --output-format csv -- python tools/physics_bench.py --steps 10 --emulate-ranks 4 > $O/tr_p4.log 2>&1 || { tail $O/tr_p4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_p4r -o t --output-format csv -- python tools/physics_bench.py --steps 10 --emulate-ranks 4 --replicated > $O/tr_p4r.log 2>&1 || { tail $O/tr_p4r.log; exit 1; }
for t in tr_r8 tr_p1 tr_p4 tr_p4r; do
  echo "== $t"; grep '^{' $O/$t.log | head -1 | cut -c1-200
  python tools/step_timeline.py $O/$t/t_kernel_trace.csv > $O/$t.timeline.txt && tail -3 $O/$t.timeline.txt
  python tools/trace_step.py $O/$t/t_kernel_trace.csv > $O/$t.step.txt && head -12 $O/$t.step.txt
done
echo rc=0
