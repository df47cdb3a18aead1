# dedup passes on the real step's target rows (N=1 and rank 0 of 8)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 8; do
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/dstep_$r -o t --output-format csv -- python tools/dedup_step_probe.py --ranks $r > gpurun_out/dstep_$r.log 2>&1 || exit 1
done
echo rc=$?
