# epilogue-feature timings (tools/epi_cost.py) of the in-tree library against tools/bin/old, alternating, same box
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 200 python tools/epi_cost.py > gpurun_out/epi_new_$i.log 2>&1 || exit 1
LLP_LIB=$GRAFT_REPO_ROOT/tools/bin/old/libllp_hip.so timeout -k 10 200 python tools/epi_cost.py > gpurun_out/epi_old_$i.log 2>&1 || exit 1
done
echo rc=$?
