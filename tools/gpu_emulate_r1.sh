# single process, rank 1's shard of a 2-rank job (offsets b0=B/2, p0=P/2), eager steps, then rank 0's
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-graph --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --emulate-ranks 2 --emulate-rank 1 ${EXTRA} > gpurun_out/emu_r1.log 2>&1 || { echo rank1 failed; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-graph --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --emulate-ranks 2 --emulate-rank 0 > gpurun_out/emu_r0.log 2>&1 || { echo rank0 failed; exit 1; }
echo rc=$?
