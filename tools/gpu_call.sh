#!/bin/bash
# GPU call recipes (replaces round 3's one-off tools/gpu_r3_call*.sh).
#
#   gpurun --timeout T -- bash tools/gpu_call.sh OUTTAG RECIPE [RECIPE ...]
#
# Runs the recipes in order, each GPU step under its own time limit; the first failing
# step ends the call (no retries).  Everything is written under gpurun_out/OUTTAG/.
# A/B recipes compare the default library with LLP_LIB=$AB_LIB (a build_lib.build_variant
# output) on the same box, interleaved.
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
LEAN="--no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32"
PROF="rocprofv3 --kernel-trace --stats --output-format csv"

fail() { echo "step failed: $1"; tail -30 "$2"; exit 1; }

for RA in "$@"; do
  R=${RA%%:*}                                 # RECIPE or RECIPE:ARGS (ARGS comma-separated)
  ARGS=$([ "$R" != "$RA" ] && echo "${RA#*:}" | tr ',' ' ')
  echo "== $RA"
  case $R in
    tests)          # the whole GPU suite
      timeout -k 10 900 $PYT tests -m gpu -q > $O/pytest_gpu.log 2>&1 || fail tests $O/pytest_gpu.log
      tail -1 $O/pytest_gpu.log ;;
    tests-sel)      # a selection: tests-sel:tests/x.py::test_a,tests/y.py
      timeout -k 10 900 $PYT $ARGS -m gpu > $O/pytest_sel.log 2>&1 || fail tests-sel $O/pytest_sel.log
      tail -1 $O/pytest_sel.log ;;
    fullsize-oracle) # the full-size oracle parity test with its printed per-tensor table (-s)
      timeout -k 10 600 $PYT -s tests/test_gpu_fullsize_oracle.py -m gpu > $O/fullsize_oracle.log 2>&1 || fail fullsize-oracle $O/fullsize_oracle.log
      grep -A14 "gradient max" $O/fullsize_oracle.log ;;
    tests-multirank)
      timeout -k 10 900 $PYT tests/test_gpu_multirank.py -q > $O/pytest_multirank.log 2>&1 || fail multirank $O/pytest_multirank.log
      tail -1 $O/pytest_multirank.log ;;
    bench)          # the default bench line (the driver's command)
      timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
      tail -c 400 $O/bench.json ;;
    bench-lean)     # the collab line alone
      timeout -k 10 300 python bench.py $LEAN > $O/bench_lean.json 2> $O/bench_lean.err || fail bench-lean $O/bench_lean.err
      cat $O/bench_lean.json ;;
    smoke)          # __graft_entry__.smoke(): one small step on cuda:0 against the oracle
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
      tail -3 $O/smoke.log ;;
    trace)          # kernel trace + stats of the collab bench (hipGraph replay)
      timeout -k 10 300 $PROF -d $O/trace -o t -- python bench.py --steps 10 --warmup 3 $LEAN > $O/trace.log 2>&1 || fail trace $O/trace.log ;;
    pmc-dominant)   # FETCH / WRITE / SQ passes on the dominant GEMM alone
      D="python bench.py --dominant-only 12 $LEAN"
      timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p --output-format csv -- $D > $O/pmc_fetch.log 2>&1 || fail pmc-fetch $O/pmc_fetch.log
      timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p --output-format csv -- $D > $O/pmc_write.log 2>&1 || fail pmc-write $O/pmc_write.log
      timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $O/pmc_sq -o p --output-format csv -- $D > $O/pmc_sq.log 2>&1 || fail pmc-sq $O/pmc_sq.log ;;
    pmc-memory)     # FETCH / WRITE passes + kernel trace of eager collab steps (memory-bound kernels)
      S="python bench.py --no-graph --steps 4 --warmup 2 --profile-kernels $LEAN"
      timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/pmcm_fetch -o run --output-format csv -- $S > $O/pmcm_fetch.log 2>&1 || fail pmcm-fetch $O/pmcm_fetch.log
      timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/pmcm_write -o run --output-format csv -- $S > $O/pmcm_write.log 2>&1 || fail pmcm-write $O/pmcm_write.log
      timeout -k 10 180 rocprofv3 --kernel-trace -d $O/pmcm_trace -o run --output-format csv -- $S > $O/pmcm_trace.log 2>&1 || fail pmcm-trace $O/pmcm_trace.log ;;
    fp32)           # the collab step in fp32 (the reference's arithmetic): bench line, trace, dominant PMC
      F32="--dtype fp32 $LEAN --no-practical-peak"
      timeout -k 10 300 python bench.py --steps 5 --warmup 2 --dtype fp32 $LEAN > $O/fp32_bench.json 2> $O/fp32_bench.err || fail fp32-bench $O/fp32_bench.err
      cat $O/fp32_bench.json
      timeout -k 10 300 $PROF -d $O/fp32_trace -o t -- python bench.py --steps 4 --warmup 2 $F32 > $O/fp32_trace.log 2>&1 || fail fp32-trace $O/fp32_trace.log
      D="python bench.py --dominant-only 6 $F32"
      timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/fp32_pmc_fetch -o p --output-format csv -- $D > $O/fp32_pmc_fetch.log 2>&1 || fail fp32-fetch $O/fp32_pmc_fetch.log
      timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/fp32_pmc_write -o p --output-format csv -- $D > $O/fp32_pmc_write.log 2>&1 || fail fp32-write $O/fp32_pmc_write.log ;;
    fp32-ab)        # fp32 collab step: default build against LLP_LIB=$AB_LIB (a build_lib.build_variant output,
                    # e.g. -DLLP_NO_L2_ORDER -> tools/bin/no_l2_order.so, the default), 3 rounds
      F32="--dtype fp32 $LEAN --no-practical-peak --steps 5 --warmup 2"
      for i in 1 2 3; do
        for L in linkless-link-prediction_amd/libllp_hip.so ${AB_LIB:-tools/bin/no_l2_order.so}; do
          LLP_LIB=$L timeout -k 10 300 python bench.py $F32 > $O/fp32_ab.tmp 2> $O/fp32_ab.err || fail fp32-ab $O/fp32_ab.err
          echo "{\"lib\": \"$L\", \"run\": $(tail -1 $O/fp32_ab.tmp)}" >> $O/fp32_ab.jsonl
        done
      done
      cut -c1-160 $O/fp32_ab.jsonl ;;
    fp32-sq)        # SQ / GRBM counters of the dominant fp32 GEMM (MFMA busy, waits, LDS)
      D="python bench.py --dominant-only 6 --dtype fp32 $LEAN --no-practical-peak"
      timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d $O/fp32_pmc_sq -o p --output-format csv -- $D > $O/fp32_pmc_sq.log 2>&1 || fail fp32-sq $O/fp32_pmc_sq.log ;;
    teacher)        # kernel trace of the SAGE teacher step (a11-a13) at the collab shape, bf16 and fp32
      for dt in bf16 fp32; do
        timeout -k 10 300 python tools/sage_bench.py --no-agg --dtype $dt --steps 10 > $O/teacher_$dt.json 2> $O/teacher_$dt.err || fail teacher-$dt $O/teacher_$dt.err
        cat $O/teacher_$dt.json
        timeout -k 10 300 $PROF -d $O/teacher_trace_$dt -o t -- python tools/sage_bench.py --no-agg --dtype $dt --steps 6 > $O/teacher_trace_$dt.log 2>&1 || fail teacher-trace $O/teacher_trace_$dt.log
      done ;;
    teacher-pmc)    # FETCH / WRITE passes of the teacher step (the aggregate's traffic inside the step)
      S="python tools/sage_bench.py --no-agg --dtype bf16 --steps 3"
      timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/tpmc_fetch -o run --output-format csv -- $S > $O/tpmc_fetch.log 2>&1 || fail tpmc-fetch $O/tpmc_fetch.log
      timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/tpmc_write -o run --output-format csv -- $S > $O/tpmc_write.log 2>&1 || fail tpmc-write $O/tpmc_write.log
      timeout -k 10 180 rocprofv3 --kernel-trace -d $O/tpmc_trace -o run --output-format csv -- $S > $O/tpmc_trace.log 2>&1 || fail tpmc-trace $O/tpmc_trace.log ;;
    sage-agg)       # every aggregate configuration, event-timed, with PMC passes
      A="python tools/sage_bench.py --agg-only --iters 10 --orders id,locality"
      timeout -k 10 180 $A > $O/sage_plan.json 2> $O/sage_plan.err || fail sage-plan $O/sage_plan.err
      timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/sage_fetch -o run --output-format csv -- $A > $O/sage_fetch.log 2>&1 || fail sage-fetch $O/sage_fetch.log
      timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $O/sage_write -o run --output-format csv -- $A > $O/sage_write.log 2>&1 || fail sage-write $O/sage_write.log ;;
    agg-ab)         # the aggregate in the teacher's order: the default library against each of $AB_LIBS
                    # (space-separated build_variant outputs), 2 interleaved rounds
      for i in 1 2; do
        for L in linkless-link-prediction_amd/libllp_hip.so ${AB_LIBS:-}; do
          LLP_LIB=$L timeout -k 10 180 python tools/sage_bench.py --agg-only --iters 20 --orders locality > $O/agg_ab.tmp 2> $O/agg_ab.err || fail agg-ab $O/agg_ab.err
          echo "{\"lib\": \"$L\", \"run\": $(tail -1 $O/agg_ab.tmp)}" >> $O/agg_ab.jsonl
        done
      done
      python tools/agg_ab_table.py $O/agg_ab.jsonl ;;
    gemm-ab)        # tools/gemm_vs_blaslt.py (GEMM_ARGS) with the default library and each of $AB_LIBS, 2 rounds
      for i in 1 2; do
        for L in linkless-link-prediction_amd/libllp_hip.so ${AB_LIBS:-}; do
          echo "# lib $L round $i" >> $O/gemm_ab.txt
          LLP_LIB=$L timeout -k 10 240 python tools/gemm_vs_blaslt.py ${GEMM_ARGS:-} >> $O/gemm_ab.txt 2> $O/gemm_ab.err || fail gemm-ab $O/gemm_ab.err
        done
      done
      cat $O/gemm_ab.txt ;;
    emulate8)       # rank 0's shard of the collab step at 8 ranks: bench line and kernel trace
      timeout -k 10 300 python bench.py --steps 20 --warmup 3 --emulate-ranks 8 > $O/emu8.json 2> $O/emu8.err || fail emu8 $O/emu8.err
      cat $O/emu8.json
      timeout -k 10 300 $PROF -d $O/emu8_trace -o t -- python bench.py --steps 10 --warmup 3 --emulate-ranks 8 > $O/emu8_trace.log 2>&1 || fail emu8-trace $O/emu8_trace.log ;;
    emulate-all)    # every rank's shard at 2, 4 and 8 ranks (per-rank time and student rows)
      for n in 2 4 8; do
        for r in $(seq 0 $((n - 1))); do
          timeout -k 10 300 python bench.py --steps 20 --warmup 3 --emulate-ranks $n --emulate-rank $r >> $O/emu_all.jsonl 2> $O/emu_all.err || fail emu-all $O/emu_all.err
        done
      done
      cat $O/emu_all.jsonl ;;
    physics)        # the physics production step, 1 rank and rank 0 of 4: bench lines and traces
      timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 > $O/phys1.json 2> $O/phys1.err || fail phys1 $O/phys1.err
      timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --emulate-ranks 4 > $O/phys4.json 2> $O/phys4.err || fail phys4 $O/phys4.err
      cat $O/phys1.json $O/phys4.json
      timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --graph > $O/phys1g.json 2> $O/phys1g.err || fail phys1g $O/phys1g.err
      timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --emulate-ranks 4 --graph > $O/phys4g.json 2> $O/phys4g.err || fail phys4g $O/phys4g.err
      cat $O/phys1g.json $O/phys4g.json
      timeout -k 10 300 $PROF -d $O/phys_t1 -o t -- python tools/physics_bench.py --steps 10 --dtype bf16 --graph > $O/phys_t1.log 2>&1 || fail phys-t1 $O/phys_t1.log
      timeout -k 10 300 $PROF -d $O/phys_t4 -o t -- python tools/physics_bench.py --steps 10 --dtype bf16 --emulate-ranks 4 --graph > $O/phys_t4.log 2>&1 || fail phys-t4 $O/phys_t4.log ;;
    physics-ab)     # sparse vs dense first student layer, graph replays, 1 rank and rank 0 of 4, twice
      for i in 1 2; do for E in "" "--emulate-ranks 4"; do for D in "" "--dense-input"; do
        timeout -k 10 300 python tools/physics_bench.py --steps 20 --dtype bf16 --graph $E $D > $O/phys_ab.tmp 2> $O/phys_ab.err || fail physics-ab $O/phys_ab.err
        echo "{\"args\": \"$E $D\", \"run\": $(head -1 $O/phys_ab.tmp)}" >> $O/phys_ab.jsonl
      done; done; done
      cut -c1-200 $O/phys_ab.jsonl ;;
    bf16-accuracy)  # paired bf16 - fp32 Hits@K over seeds (tools/bf16_accuracy.py)
      timeout -k 10 1000 python tools/bf16_accuracy.py ${ACC_ARGS:-} > $O/bf16_accuracy.jsonl 2> $O/bf16_accuracy.err || fail bf16-accuracy $O/bf16_accuracy.err
      tail -5 $O/bf16_accuracy.jsonl ;;
    ab)             # same-box A/B of AB_SCRIPT (default: the lean collab bench) against LLP_LIB=$AB_LIB (default:
                    # the same library) running AB_SCRIPT_VAR (default: AB_SCRIPT), 3 rounds
      S=${AB_SCRIPT:-"python bench.py $LEAN"}
      SV=${AB_SCRIPT_VAR:-$S}
      for i in 1 2 3; do
        timeout -k 10 300 $S > $O/ab_base_$i.json 2> $O/ab_base_$i.err || fail ab-base $O/ab_base_$i.err
        LLP_LIB=${AB_LIB:-linkless-link-prediction_amd/libllp_hip.so} timeout -k 10 300 $SV > $O/ab_var_$i.json 2> $O/ab_var_$i.err || fail ab-var $O/ab_var_$i.err
      done
      tail -n 1 $O/ab_base_*.json $O/ab_var_*.json ;;
    *)
      echo "unknown recipe $R"; exit 2 ;;
  esac
done
echo rc=0
