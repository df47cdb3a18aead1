# Round 3, fourth GPU call: bf16-vs-fp32 training accuracy at scaled collab (two seeds),
# the counters this rocprofv3 lists (DRAM-side ones), the bench line with the fp32 leg.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/c4_counters.txt 2>&1 || true
grep -i -E "dram|hbm|mall|EA0_RD|TCC_EA" gpurun_out/c4_counters.txt | head -40
timeout -k 10 500 python -u tools/bf16_accuracy.py --seeds 2 --epochs 8 > gpurun_out/c4_bf16_acc.json 2> gpurun_out/c4_bf16_acc.err || { echo "bf16 accuracy failed"; tail -20 gpurun_out/c4_bf16_acc.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/c4_bf16_acc.json'):
    d=json.loads(l)
    print({k: {s: round(v*100, 3) for s, v in x.items()} for k, x in d['bf16_minus_fp32'].items()}, {dt: round(r['seconds'],1) for dt, r in d['runs'].items()}, d['final']['fp32']['Hits@20'])
"
timeout -k 10 700 python bench.py > gpurun_out/c4_bench1.json 2> gpurun_out/c4_bench1.err || { echo "bench failed"; tail -20 gpurun_out/c4_bench1.err; exit 1; }
python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/c4_bench1.json') if l.startswith('{')][0]
print(d['ms_per_step'], d['value'], d.get('fp32_step'), [ (x['dtype'],x['F'],round(x['ms']*1e3,1),round(x['frac'],3)) for x in d['sage_aggregate']])
"
echo rc=0
