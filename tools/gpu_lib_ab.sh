# A/B of the in-tree library against another build (tools/bin/old/libllp_hip.so, tools/build_old_lib.sh) on the collab step
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --no-shard8 --steps 50"
for i in 1 2 3; do
timeout -k 10 300 $B > gpurun_out/ab_new_$i.json 2>&1 || exit 1
LLP_LIB=$GRAFT_REPO_ROOT/tools/bin/old/libllp_hip.so timeout -k 10 300 $B > gpurun_out/ab_old_$i.json 2>&1 || exit 1
done
echo rc=$?
