export TMPDIR=/tmp
OUT=gpurun_out/r5h
mkdir -p $OUT
timeout -k 10 300 python -u tools/kernel_bench.py gemm_swin > $OUT/kb.jsonl 2> $OUT/kb.err || { echo "STOP kb"; tail $OUT/kb.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/kb.jsonl'):
    d=json.loads(l)
    if 'kernel' in d: print(d['kernel'], d['config'].split(' bf16')[0], d['ms'], d['achieved'])
"
for g in 1 0 1 0; do
  LCI_HIP_GEMM=$g timeout -k 10 600 python -u bench.py --workload swin_p2_128 --steps 10 --warmup 3 > $OUT/c3_$g.json 2> $OUT/c3_$g.err || { echo "STOP c3 $g"; tail -3 $OUT/c3_$g.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c3_$g.json').read().strip().splitlines()[-1]); print('C3 HIP_GEMM=$g', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items() if 'gemm' in k or 'linear' in k})"
done
