# bf16 vs fp32 curves with 2,000 planted communities (scaled collab: ~5 same-community pairs among the 10,000 negatives)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/bf16_accuracy.py --seeds 3 --epochs 48 --eval-every 8 --communities 2000 > gpurun_out/c6_bf16_acc.json 2> gpurun_out/c6_bf16_acc.err || { echo "failed"; tail -20 gpurun_out/c6_bf16_acc.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/c6_bf16_acc.json'):
    d=json.loads(l)
    for dt in ('fp32','bf16'):
        print(dt, [(h['epoch'], round(h['loss'],4), round(100*h['hits']['Hits@20']['test'],2), round(100*h['hits']['Hits@50']['test'],2), round(100*h['hits']['Hits@20']['valid'],2)) for h in d['runs'][dt]['history']])
"
echo rc=0
