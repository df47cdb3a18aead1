# A/B of the second-stream overlap modes (LLP_OVERLAP bit mask) on the collab bench
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --steps 30"
for i in 1 2; do
for m in ${MODES:-0 1 2 3 6 7}; do
timeout -k 10 300 env LLP_OVERLAP=$m $B > gpurun_out/ab_${m}_$i.json 2> gpurun_out/ab_${m}_$i.err || exit 1
done
done
echo rc=$?
