# SQ / GRBM counters of the dominant GEMM launch (bench --dominant-only), plain (4) vs staggered (6) q64
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
for v in 4 6; do
LLP_GEMM_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_sq_$v -o run --output-format csv -- python bench.py --dominant-only 10 --no-cpu-baseline --no-eval --no-sage > gpurun_out/pmc_sq_$v.log 2>&1 || exit 1
done
echo rc=$?
