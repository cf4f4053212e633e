export TMPDIR=/tmp
OUT=gpurun_out/r5j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_linear_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/test.log 2>&1 || { echo "STOP test"; tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
timeout -k 10 300 python -u tools/kernel_bench.py gemm > $OUT/kb.jsonl 2> $OUT/kb.err || { echo "STOP kb"; tail $OUT/kb.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/kb.jsonl'):
    d=json.loads(l)
    if 'kernel' in d: print(d['kernel'], d['config'].split(' bf16')[0], d['ms'], d['achieved'])
"
