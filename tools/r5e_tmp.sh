export TMPDIR=/tmp
OUT=gpurun_out/r5e
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "STOP gputest"; tail -30 $OUT/gputest.log; exit 1; }
tail -2 $OUT/gputest.log
timeout -k 10 300 python -u tools/kernel_bench.py gemm mlp > $OUT/kb.jsonl 2> $OUT/kb.err || { echo "STOP kb"; tail $OUT/kb.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r5e/kb.jsonl'):
    d = json.loads(l)
    if 'kernel' in d: print(d['kernel'], d['config'].split(' bf16')[0], d['ms'], d['achieved'])
PY
timeout -k 10 600 python bench.py --no-secondary > $OUT/bench.json 2> $OUT/bench.err || { echo "STOP bench"; tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('METRIC', d['value'], d['ms_per_step'], d['roofline']['frac']); print({k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 1})"
timeout -k 10 600 python bench.py --workload vit_mamba_p2_256 --steps 5 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err || { echo "STOP c5"; tail -3 $OUT/c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c5.json').read().strip().splitlines()[-1]); print('C5', d['value'], d['ms_per_step']); print({k: v['ms_per_step'] for k, v in d['kernels'].items() if v['ms_per_step'] > 5})"
