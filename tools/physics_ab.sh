#!/bin/bash
# Same-box A/B of tools/physics_bench.py --graph (bf16) between the default engine and the
# engine switches in $VAR_ARGS (and/or the library $VAR_LIB, a build_lib.build_variant output),
# at 1 rank and rank 0 of 4, 3 interleaved rounds.
#   gpurun -- bash tools/physics_ab.sh OUTTAG "--main-sampler"
#   gpurun -- 'VAR_LIB=tools/bin/x.so bash tools/physics_ab.sh OUTTAG ""'
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
VAR_ARGS=$2
mkdir -p "$O"
B="python tools/physics_bench.py --steps 40 --warmup 3 --dtype bf16 --graph"
for i in 1 2 3; do
  for E in "--emulate-ranks 4" ""; do
    for V in base var; do
      A=$([ $V = var ] && echo "$VAR_ARGS")
      L=$([ $V = var ] && [ -n "$VAR_LIB" ] && echo "$VAR_LIB" || echo linkless-link-prediction_amd/libllp_hip.so)
      LLP_LIB=$L timeout -k 10 300 $B $E $A > $O/run.tmp 2> $O/run.err || { tail -20 $O/run.err; exit 1; }
      echo "{\"round\": $i, \"ranks\": \"$E\", \"side\": \"$V\", \"run\": $(grep -m1 "^{" $O/run.tmp)}" >> $O/ab.jsonl
    done
  done
done
python - "$O/ab.jsonl" <<'EOF'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
for ranks in ("--emulate-ranks 4", ""):
    for side in ("base", "var"):
        ms = [round(r["run"]["ms_per_step"], 4) for r in rows if r["ranks"] == ranks and r["side"] == side]
        print(f"{'rank 0 of 4' if ranks else '1 rank':12s} {side:4s} {ms}")
EOF
echo rc=0
