# FETCH_SIZE / WRITE_SIZE and SQ counters of the P-shape weight-gradient GEMM, tile-major (10) vs split-major (2)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for v in 10 2; do
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tnpmc_f$v -o run --output-format csv -- python tools/tn_one.py $v 603032 1024 1024 > gpurun_out/tnpmc_f$v.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tnpmc_w$v -o run --output-format csv -- python tools/tn_one.py $v 603032 1024 1024 > gpurun_out/tnpmc_w$v.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/tnpmc_s$v -o run --output-format csv -- python tools/tn_one.py $v 603032 1024 1024 > gpurun_out/tnpmc_s$v.log 2>&1 || exit 1
done
echo rc=$?
