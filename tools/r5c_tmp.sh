export TMPDIR=/tmp
OUT=gpurun_out/r5c
mkdir -p $OUT
for p in 1 0; do
  LCI_GEMM_PROBE=$p timeout -k 10 300 python -u tools/kernel_bench.py gemm > $OUT/gemm_p$p.jsonl 2> $OUT/gemm_p$p.err || { echo "STOP gemm p$p"; exit 1; }
done
python3 - <<'PY'
import json
for p in (1, 0):
    for l in open(f'gpurun_out/r5c/gemm_p{p}.jsonl'):
        d = json.loads(l)
        if d['kernel'].startswith('gemm_bt') or p == 0: print(f"probe{p}", d['kernel'], d['config'].split(' bf16')[0], d['ms'], d['achieved'])
PY
bash tools/profile_r5.sh r5 metric c3 fft || exit 1
timeout -k 10 600 python bench.py --workload vit_mamba_p2_256 --steps 5 --warmup 2 > $OUT/c5.json 2> $OUT/c5.err || { echo "STOP c5"; tail -3 $OUT/c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c5.json').read().strip().splitlines()[-1]); print('C5', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']); print({k: v for k, v in d['kernels'].items() if 'scan' in k})"
