# A/B of an engine environment knob on the collab step: ENV_A vs ENV_B (e.g. LLP_SEGMENT_FUSED=0 / =1), 3 rounds
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --no-shard8 --steps 50"
for i in 1 2 3; do
env $ENV_A timeout -k 10 300 $B > gpurun_out/ab_old_$i.json 2>&1 || exit 1
env $ENV_B timeout -k 10 300 $B > gpurun_out/ab_new_$i.json 2>&1 || exit 1
done
echo rc=$?
