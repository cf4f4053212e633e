export TMPDIR=/tmp
OUT=gpurun_out/r5d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $OUT/test.log 2>&1 || { echo "STOP test"; tail -20 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
for p in 2 3 0; do
  LCI_GEMM_PROBE=$p timeout -k 10 300 python -u tools/kernel_bench.py gemm > $OUT/gemm_p$p.jsonl 2> $OUT/gemm_p$p.err || { echo "STOP gemm"; tail $OUT/gemm_p$p.err; exit 1; }
done
python3 - <<'PY'
import json
for p in (2, 3, 0):
    for l in open(f'gpurun_out/r5d/gemm_p{p}.jsonl'):
        d = json.loads(l)
        if 'kernel' in d and (p == 0 or d['kernel'].startswith('gemm_bt')): print(p, d['kernel'], d['config'].split(' bf16')[0], d['ms'], d['achieved'])
PY
