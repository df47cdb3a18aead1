# round-3 profiles: default bench line, kernel trace + stats, dominant-kernel PMC (FETCH, WRITE, SQ)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
T="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o t --output-format csv -- $T > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
D="python bench.py --dominant-only 12 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p --output-format csv -- $D > $O/pmc_fetch.log 2>&1 || { tail $O/pmc_fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p --output-format csv -- $D > $O/pmc_write.log 2>&1 || { tail $O/pmc_write.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $O/pmc_sq -o p --output-format csv -- $D > $O/pmc_sq.log 2>&1 || { tail $O/pmc_sq.log; exit 1; }
grep dominant_rows $O/pmc_sq.log
echo rc=0
