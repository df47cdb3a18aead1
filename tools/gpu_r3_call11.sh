# persistent NT GEMM: bit-identity tests + the whole suite; step A/B against pp8 (3 interleaved rounds)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_kernels.py -m gpu -k "persistent" > gpurun_out/c11_persist.log 2>&1 || { echo "persistent tests failed"; tail -30 gpurun_out/c11_persist.log; exit 1; }
tail -1 gpurun_out/c11_persist.log
true

B="python bench.py --no-eval --no-sage --no-physics --no-cpu-baseline --no-shard8 --no-fp32 --steps 50"
for i in 1 2 3; do
LLP_LIB=tools/bin/libllp_hip_pp8p_drain.so timeout -k 10 300 $B > gpurun_out/c11_old_$i.json 2>&1 || exit 1
timeout -k 10 300 $B > gpurun_out/c11_new_$i.json 2>&1 || exit 1
done
for f in gpurun_out/c11_old_*.json gpurun_out/c11_new_*.json; do python -c "
import json,sys
d=[json.loads(l) for l in open('$f') if l.startswith('{')][0]
print('$f', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],4), round(d['roofline']['achieved'],1))"; done
T="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eval --no-sage --no-physics --no-shard8 --no-fp32"
LLP_LIB=tools/bin/libllp_hip_pp8p_drain.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c11_tr_old -o t --output-format csv -- $T > gpurun_out/c11_tr_old.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c11_tr_new -o t --output-format csv -- $T > gpurun_out/c11_tr_new.log 2>&1 || exit 1
python tools/trace_summary.py gpurun_out/c11_tr_old gpurun_out/c11_tr_new -k gemm_nt > gpurun_out/c11_gemm_ab.txt || exit 1
cat gpurun_out/c11_gemm_ab.txt
echo rc=0
