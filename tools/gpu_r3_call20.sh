# practical MFMA peak beside the dominant GEMM: the default bench line
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/c20
mkdir -p $O
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value']); print(json.dumps(d['roofline']))"
echo rc=0
