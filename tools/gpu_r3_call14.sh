# physics full-batch step, bf16: kernel traces at 1 rank and rank 0 of 4 (sharded / replicated student)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c14
mkdir -p $O
P="python tools/physics_bench.py --steps 10 --dtype bf16"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_p1 -o t --output-format csv -- $P > $O/tr_p1.log 2>&1 || { tail $O/tr_p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_p4 -o t --output-format csv -- $P --emulate-ranks 4 > $O/tr_p4.log 2>&1 || { tail $O/tr_p4.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_p4r -o t --output-format csv -- $P --emulate-ranks 4 --replicated > $O/tr_p4r.log 2>&1 || { tail $O/tr_p4r.log; exit 1; }
for t in tr_p1 tr_p4 tr_p4r; do
  echo "== $t"; grep '^{' $O/$t.log | head -1 | cut -c1-200
  python tools/step_timeline.py $O/$t/t_kernel_trace.csv > $O/$t.timeline.txt && tail -1 $O/$t.timeline.txt
  python tools/trace_step.py $O/$t/t_kernel_trace.csv > $O/$t.step.txt && head -16 $O/$t.step.txt
done
echo rc=0
