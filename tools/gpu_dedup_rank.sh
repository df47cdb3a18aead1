# dedup passes: counting path with the atomic cursor (default) vs the rank variant (LLP_DEDUP_RANK=1)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 0 1; do
LLP_DEDUP_RANK=$v timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/dedup_$v -o t --output-format csv -- python tools/dedup_probe.py > gpurun_out/dedup_$v.log 2>&1 || exit 1
done
LLP_DEDUP_RANK=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dedup or unique or segments" > gpurun_out/pytest_dedup.log 2>&1 || { echo tests failed; exit 1; }
echo rc=$?
