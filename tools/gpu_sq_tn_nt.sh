# SQ counters of the P-shape weight-gradient TN GEMM and the dominant NT GEMM (one pass each)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
timeout -s KILL 90 rocprofv3 --pmc $C -d gpurun_out/sq_tn -o run --output-format csv -- python tools/tn_one.py 5 603032 1024 1024 > gpurun_out/sq_tn.log 2>&1 || exit 1
#timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/sq_nt -o run --output-format csv -- python bench.py --dominant-only 10 --no-cpu-baseline --no-eval --no-sage > gpurun_out/sq_nt.log 2>&1 || exit 1
C2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS"
timeout -s KILL 90 rocprofv3 --pmc $C2 -d gpurun_out/sq2_tn -o run --output-format csv -- python tools/tn_one.py 5 603032 1024 1024 > gpurun_out/sq2_tn.log 2>&1 || exit 1
#timeout -s KILL 120 rocprofv3 --pmc $C2 -d gpurun_out/sq2_nt -o run --output-format csv -- python bench.py --dominant-only 10 --no-cpu-baseline --no-eval --no-sage > gpurun_out/sq2_nt.log 2>&1 || exit 1
echo rc=$?
